"""Backbone / RPN convolution on libtlod's MFMA implicit-GEMM kernels.

``Conv2d`` is a drop-in for the ``nn.Conv2d`` modules inside the reference's
``RCNN_base`` (torchvision vgg16().features, lib/DAF/vgg16.py:49) and ``RPN_Conv``
(lib/model/rpn/rpn.py:28): same parameters, same state_dict keys, same default
shapes.  ``relu=True`` fuses the following ``nn.ReLU`` into the kernel epilogue (the
backward then applies the ReLU mask from the saved output).

Forward, input-gradient and weight-gradient all run in libtlod (tlod_conv_*_f32).
Weight gradient is only computed when the weight requires grad, input gradient only
when the input does (conv3_1 of VGG16 needs no dgrad: its input comes from frozen
layers, lib/DAF/vgg16.py:52-53).
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .grads import grad_out


# Optional launch timing (bench.py): list of (start_event, end_event, flops, kind, shape)
# or None; shape = (N, Cin, H, W, Cout, KS).
PROFILE = None


def _timed(kind, shape, fn, math="f32"):
    """Run one launch; under bench.py's PROFILE also record HIP events around it on the
    launch stream.  kind: fwd / dgrad / wgrad with shape (N, Cin, H, W, Cout, KS), or
    gemm (tlod.linear) with shape (M, N, K)."""
    if PROFILE is None:
        return fn()
    if kind == "gemm":
        M, Nn, K = shape
        flops = 2.0 * M * Nn * K
    else:
        N, Cin, H, W, Cout, KS = shape
        flops = 2.0 * N * H * W * Cout * Cin * KS * KS
    kind = f"{kind}/{math}"
    # events from bench.py's pre-created pool when it has one (creating two events per
    # launch cost the host ~10 us per launch inside the timed region)
    pool = getattr(PROFILE, "pool", None)
    if pool:
        s, e = pool.pop()
    else:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    r = fn()
    e.record()
    PROFILE.append((s, e, flops, kind, shape))
    return r


MATHS = ("f32", "bf16x6", "bf16x3")


def conv_math():
    """Arithmetic of the 3x3 fwd/dgrad convolutions (env TLOD_CONV_MATH):
      "bf16x6" (default): f32 operands split exactly into 3 bf16 terms, the 6 products down
               to 2^-16 relative on the bf16 MFMA, f32 accumulation — f32-level error (the
               same normwise ~1e-7 vs fp64 as the f32-input MFMA; tests/test_conv_bs_gpu.py);
      "f32"  : the f32-input MFMA (exact f32 products);
      "bf16x3": 3 products (~5e-6 normwise), opt-in.
    The 3x3 weight gradients follow it too (override: TLOD_WGRAD_MATH); 1x1 convs with >= 64
    input and output channels (the ResNet bottlenecks, DA heads) run their forward / input
    gradient on the split-bf16 conv GEMM too (_gemm1x1), narrower ones (RPN heads) on the
    f32-input MFMA."""
    m = _lib.env("TLOD_CONV_MATH", "bf16x6")
    if m not in MATHS:
        raise ValueError(f"TLOD_CONV_MATH={m!r}: expected one of {MATHS}")
    return m


def _bs(KS, math):
    return KS == 3 and math != "f32"


def _wgrad_1x1_bs(KS, math):
    """1x1 weight gradients (RPN cls/bbox heads, image-DA conv) under a split-bf16 math run
    on tlod_conv_wgrad_bs_f32 with KS = 1 (measured 0.135 vs 0.23 ms per step on the f32
    kernel); their forward / input gradient stay on the f32-MFMA kernels, which beat
    per-image split-bf16 GEMMs at these sizes (0.26 vs 0.41 ms per step)."""
    return KS == 1 and math != "f32"


def _gemm_conv(KS, math, out_channels):
    """3x3 split-bf16 convs with >= 256 output channels run as an implicit GEMM over
    flattened pixels (tlod_conv3x3_gemm_bs_f32, 256x256 tiles); narrower ones keep the
    patch-staged kernel (tlod_conv_fwd_bs_f32).  Opt-in (TLOD_CONV_GEMM=1): measured equal
    to the patch-staged kernel in the DAF step (conv3_3 fwd 0.558 vs 0.553 ms)."""
    return (_bs(KS, math) and out_channels >= 256
            and _lib.env("TLOD_CONV_GEMM", "0") != "0")


def _gemm1x1(KS, math, cin, cout):
    """1x1 convs under a split-bf16 math with >= 64 channels on one side and >= 16 on the
    other run their forward / input gradient as per-image GEMMs on the split-bf16 conv GEMM
    (tlod_conv1x1_gemm_bs_f32: W (Cout x Cin) times the image's (Cin x HW) map, 64/128/256-row
    tiles by Cout, the folded-BN / residual / ReLU epilogue) — the ResNet bottlenecks, the DA
    image heads and (round 4) the RPN cls / bbox heads (18 / 36 outputs: a 64-row tile
    mostly padding still beats the f32-input MFMA kernel's 6.6 TF); TLOD_CONV1X1_BS=0 keeps
    them on the f32-input MFMA kernel."""
    return (KS == 1 and math != "f32" and max(cin, cout) >= 64
            and min(cin, cout) >= int(_lib.env("TLOD_CONV1X1_MIN", "16"))
            and _lib.env("TLOD_CONV1X1_BS", "1") != "0")


def _conv_gemm(x, w, w_layout, bias, relu, scale, residual, Cout, math, kind, KS=3, mask=None,
               wscale=None):
    N, Cin, H, W = x.shape
    y = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device)
    b = bias.detach().contiguous() if bias is not None else None
    sc = scale.detach().contiguous() if scale is not None else None
    res = residual.detach().contiguous() if residual is not None else None
    if res is not None:
        assert res.shape == y.shape, (res.shape, y.shape)
    L = _lib.lib()
    nprod = 6 if math == "bf16x6" else 3
    wsb, fn, name = ((L.tlod_conv3x3_gemm_bs_workspace_bytes, L.tlod_conv3x3_gemm_bs_f32,
                      "conv3x3_gemm_bs") if KS == 3 else
                     (L.tlod_conv1x1_gemm_bs_workspace_bytes, L.tlod_conv1x1_gemm_bs_f32,
                      "conv1x1_gemm_bs"))
    ws = _lib.workspace(wsb(N, Cin, H, W, Cout, w_layout, nprod), x.device, "conv")
    shape = (N, Cin, H, W, Cout, KS) if kind == "fwd" else (N, Cout, H, W, Cin, KS)
    if mask is not None or wscale is not None:
        # 1x1 only (tlod_conv1x1_gemm_bs_ex_f32): y *= (mask > 0) last; the weight's output
        # channels scaled by wscale as it is staged (dgrad layout)
        assert KS == 1 and (mask is None or mask.shape == y.shape), (KS, y.shape)
        mk = mask.detach().contiguous() if mask is not None else None
        wsc = wscale.detach().contiguous() if wscale is not None else None
        _timed(kind, shape, lambda: _lib.check(
            L.tlod_conv1x1_gemm_bs_ex_f32(_lib.ptr(x), _lib.ptr(w), w_layout, _lib.ptr(sc),
                                          _lib.ptr(b), _lib.ptr(res), _lib.ptr(mk), _lib.ptr(wsc),
                                          _lib.ptr(y), N, Cin, H, W, Cout, int(relu), nprod,
                                          _lib.ptr(ws), ws.numel(), _lib.stream_of(x)),
            "conv1x1_gemm_bs_ex"), math)
        return y
    _timed(kind, shape, lambda: _lib.check(
        fn(_lib.ptr(x), _lib.ptr(w), w_layout, _lib.ptr(sc), _lib.ptr(b), _lib.ptr(res),
           _lib.ptr(y), N, Cin, H, W, Cout, int(relu), nprod, _lib.ptr(ws), ws.numel(),
           _lib.stream_of(x)), name),
        math)
    return y


# Writes to frozen weights that bypass torch's version counter (the data-parallel start-up
# broadcast, tlod.dist, writes through .data) bump this, so the cached packs are remade.
_EXTERNAL_WRITES = [0]


def weights_updated():
    """Called after a write to parameters that did not bump their version counters."""
    _EXTERNAL_WRITES[0] += 1


# Generation of the set of packs that tlod.optim.FusedSGDClip keeps current: bumped when a
# pack of a weight it owns is (re)made, so the optimizer rebuilds its tile table.
PACK_GEN = [0]


def pack_bs(weight, dgrad, scale=None):
    """Pre-split bf16 planes of a 3x3 weight for the split-bf16 fwd (dgrad=0) / dgrad (1);
    scale (Cout, optional): of weight[co] * scale[co] (a frozen BatchNorm's scale after the
    conv).  Cached on the tensor per (dgrad, scale) for frozen weights (requires_grad False:
    conv1/conv2 of VGG16, the fixed ResNet blocks) and for weights a FusedSGDClip owns
    (`_tlod_pack_owner`: its update writes the new packs in the same kernel,
    tlod_sgd_clip_pack_f32); valid per (storage, version, external writes) — an in-place load
    bumps the version, a write that bypasses it (the data-parallel broadcast) calls
    weights_updated().  Other trainable weights are repacked every call."""
    owned = weight.requires_grad and getattr(weight, "_tlod_pack_owner", False)
    if weight.requires_grad and (not owned or (scale is not None and not dgrad)):
        return _pack_bs(weight, dgrad, scale)  # (the fused update keeps no scaled fwd pack)
    packs = getattr(weight, "_tlod_packs", None)  # lives and dies with the tensor
    if packs is None:
        packs = weight._tlod_packs = {}
    vkey = (bool(dgrad), None if scale is None else (scale.data_ptr(), scale._version))
    key = (weight.data_ptr(), weight._version, _EXTERNAL_WRITES[0])
    hit = packs.get(vkey)
    if hit is None or hit[0] != key:
        if scale is not None:  # one scaled variant per weight (the fused update's tile has one)
            for k in [k for k in packs if k[1] is not None]:
                del packs[k]
        hit = (key, _pack_bs(weight, dgrad, scale), scale)
        packs[vkey] = hit
        if owned:
            PACK_GEN[0] += 1
    return hit[1]


def _pack_bs(weight, dgrad, scale=None):
    """scale (Cout, optional): pack weight[co] * scale[co] (tlod_conv_pack_bs_ex)."""
    Cout, Cin, KS, _ = weight.shape
    L = _lib.lib()
    p = torch.empty(L.tlod_conv_pack_bs_bytes(Cout, Cin, KS, int(dgrad)), dtype=torch.uint8,
                    device=weight.device)
    sc = scale.detach().contiguous() if scale is not None else None
    _lib.check(L.tlod_conv_pack_bs_ex(_lib.ptr(weight.detach().contiguous()), _lib.ptr(sc), Cout,
                                      Cin, KS, int(dgrad), _lib.ptr(p), _lib.stream_of(weight)),
               "pack_bs")
    return p


def _check(x, w):
    _lib.require_cuda(x, w)
    if x.dtype != torch.float32 or w.dtype != torch.float32:
        raise TypeError("tlod conv computes in fp32 (the reference's dtype)")


def pack_fwd(weight):
    Cout, Cin, KS, _ = weight.shape
    wk = torch.empty((Cin * KS * KS, Cout), dtype=torch.float32, device=weight.device)
    _lib.check(_lib.lib().tlod_conv_pack_fwd_f32(_lib.ptr(weight.detach().contiguous()), Cout,
                                                 Cin, KS, _lib.ptr(wk), _lib.stream_of(weight)),
               "conv_pack_fwd")
    return wk


def pack_dgrad(weight):
    Cout, Cin, KS, _ = weight.shape
    wd = torch.empty((Cout * KS * KS, Cin), dtype=torch.float32, device=weight.device)
    _lib.check(_lib.lib().tlod_conv_pack_dgrad_f32(_lib.ptr(weight.detach().contiguous()), Cout,
                                                   Cin, KS, _lib.ptr(wd), _lib.stream_of(weight)),
               "conv_pack_dgrad")
    return wd


def conv_fwd(x, weight, bias=None, relu=False, wk=None, scale=None, residual=None, math=None):
    """y = act(conv(x, weight) * scale + bias + residual) (tlod_conv_fwd_ex_f32, or
    tlod_conv_fwd_bs_f32 for 3x3 under a split-bf16 math; wk: the matching pack)."""
    _check(x, weight)
    x = x.contiguous()
    N, Cin, H, W = x.shape
    Cout, _, KS, _ = weight.shape
    math = conv_math() if math is None else math
    if KS == 3 and Cin <= 4 and scale is None and residual is None:
        return _conv_direct(x, weight, bias, relu)
    if _gemm_conv(KS, math, Cout):
        return _conv_gemm(x, weight.detach().contiguous(), 0, bias, relu, scale, residual, Cout,
                          math, "fwd")
    if _gemm1x1(KS, math, Cin, Cout):
        return _conv_gemm(x, weight.detach().contiguous(), 0, bias, relu, scale, residual, Cout,
                          math, "fwd", KS=1)
    if _bs(KS, math):
        return _conv_bs(x, pack_bs(weight, False) if wk is None else wk, bias, relu, scale,
                        residual, Cout, KS, math, "fwd")
    wk = pack_fwd(weight) if wk is None else wk
    y = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device)
    b = bias.detach().contiguous() if bias is not None else None
    sc = scale.detach().contiguous() if scale is not None else None
    res = residual.detach().contiguous() if residual is not None else None
    if res is not None:
        assert res.shape == y.shape, (res.shape, y.shape)
    L = _lib.lib()
    ws = _lib.workspace(L.tlod_conv_fwd_workspace_bytes(N, Cin, H, W, Cout, KS), x.device, "conv")
    _timed("fwd", (N, Cin, H, W, Cout, KS), lambda: _lib.check(
        L.tlod_conv_fwd_ex_f32(_lib.ptr(x), _lib.ptr(wk), _lib.ptr(sc), _lib.ptr(b),
                               _lib.ptr(res), _lib.ptr(y), N, Cin, H, W, Cout, KS, int(relu),
                               _lib.ptr(ws), ws.numel(), _lib.stream_of(x)), "conv_fwd"))
    return y


def _conv_direct(x, weight, bias, relu):
    """3x3 convs with <= 4 input channels (VGG16 conv1_1 on the image): direct f32 FMA
    kernel, one thread per output pixel (tlod_conv3x3_direct_f32) — the implicit GEMM would
    pad K = 27 to a 72-deep chunk pair."""
    N, Cin, H, W = x.shape
    Cout = weight.shape[0]
    y = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device)
    b = bias.detach().contiguous() if bias is not None else None
    _timed("fwd", (N, Cin, H, W, Cout, 3), lambda: _lib.check(
        _lib.lib().tlod_conv3x3_direct_f32(_lib.ptr(x), _lib.ptr(weight.detach().contiguous()),
                                           _lib.ptr(b), _lib.ptr(y), N, Cin, H, W, Cout, int(relu),
                                           _lib.stream_of(x)), "conv3x3_direct"), "f32")
    return y


def _conv_bs(x, wp, bias, relu, scale, residual, Cout, KS, math, kind):
    N, Cin, H, W = x.shape
    y = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device)
    b = bias.detach().contiguous() if bias is not None else None
    sc = scale.detach().contiguous() if scale is not None else None
    res = residual.detach().contiguous() if residual is not None else None
    L = _lib.lib()
    nprod = 6 if math == "bf16x6" else 3
    ws = _lib.workspace(L.tlod_conv_fwd_bs_workspace_bytes(N, Cin, H, W, Cout, KS, nprod), x.device,
                        "conv")
    shape = (N, Cin, H, W, Cout, KS) if kind == "fwd" else (N, Cout, H, W, Cin, KS)
    _timed(kind, shape, lambda: _lib.check(
        L.tlod_conv_fwd_bs_f32(_lib.ptr(x), _lib.ptr(wp), _lib.ptr(sc), _lib.ptr(b), _lib.ptr(res),
                               _lib.ptr(y), N, Cin, H, W, Cout, KS, int(relu), nprod, _lib.ptr(ws),
                               ws.numel(), _lib.stream_of(x)), "conv_fwd_bs"), math)
    return y


def conv_dgrad(g, weight, wd=None, math=None, mask=None, residual=None, wscale=None):
    """Input gradient.  mask (the conv's input, when that is the previous conv's ReLU output):
    on the split-bf16 3x3 path and the split-bf16 1x1 GEMM the result is dx * (mask > 0) — the
    previous layer's ReLU backward done in this epilogue (tlod_conv_dgrad_bs_mask_f32,
    tlod_conv1x1_gemm_bs_ex_f32) — and it is tagged so that layer's backward skips its own pass
    (ConvFunction, ConvBNFunction); other paths ignore mask.  residual (1x1 GEMM path, or
    added here otherwise): a gradient summed into dx before the mask (a bottleneck's identity
    shortcut).  wscale (Cout, optional): the gradient through weight * wscale[co] (a frozen
    BatchNorm's scale after the conv) — applied as the 1x1 GEMM stages the weight or by the
    3x3 pack, not as a pass over the weight."""
    g = g.contiguous()
    N, Cout, H, W = g.shape
    _, Cin, KS, _ = weight.shape
    math = conv_math() if math is None else math
    if _gemm1x1(KS, math, Cout, Cin) and (mask is not None or residual is not None or
                                          wscale is not None):
        dx = _conv_gemm(g, weight.detach().contiguous(), 1, None, False, None, residual, Cin,
                        math, "dgrad", KS=1, mask=mask, wscale=wscale)
        if mask is not None:
            dx._tlod_relu_masked = (mask.data_ptr(), dx.data_ptr(), dx._version)
            STATS["masked_dgrad"] += 1
        return dx
    if wscale is not None:
        if _bs(KS, math) and not _gemm_conv(KS, math, Cin) and wd is None:
            wd = pack_bs(weight, True, wscale)
        else:
            weight = weight.detach() * wscale.view(-1, 1, 1, 1)
            wd = None
    if residual is not None:
        return conv_dgrad(g, weight, wd, math).add_(residual)
    if mask is not None and _bs(KS, math) and not _gemm_conv(KS, math, Cin):
        return _conv_dgrad_mask(g, pack_bs(weight, True) if wd is None else wd, mask, Cin, math)
    if _gemm_conv(KS, math, Cin):
        return _conv_gemm(g, pack_dgrad(weight), 1, None, False, None, None, Cin, math, "dgrad")
    if _gemm1x1(KS, math, Cout, Cin):
        # dx = W^T g: the (Cout, Cin) weight read as the M-contiguous (M = Cin, K = Cout) operand
        return _conv_gemm(g, weight.detach().contiguous(), 1, None, False, None, None, Cin, math,
                          "dgrad", KS=1)
    if _bs(KS, math):
        # dgrad = the forward form over dy with the transposed, flipped pack
        return _conv_bs(g, pack_bs(weight, True) if wd is None else wd, None, False, None, None,
                        Cin, KS, math, "dgrad")
    wd = pack_dgrad(weight) if wd is None else wd
    dx = torch.empty((N, Cin, H, W), dtype=torch.float32, device=g.device)
    L = _lib.lib()
    ws = _lib.workspace(L.tlod_conv_dgrad_workspace_bytes(N, Cin, H, W, Cout, KS), g.device, "conv")
    _timed("dgrad", (N, Cin, H, W, Cout, KS), lambda: _lib.check(
        L.tlod_conv_dgrad_f32(_lib.ptr(g), _lib.ptr(wd), _lib.ptr(dx), N, Cin, H, W, Cout, KS,
                              _lib.ptr(ws), ws.numel(), _lib.stream_of(g)), "conv_dgrad"))
    return dx


STATS = {"masked_dgrad": 0, "relu_bwd_skipped": 0}  # fused ReLU-backward counters (tests)


def _conv_dgrad_mask(g, wp, mask, Cin, math):
    N, Cout, H, W = g.shape
    mask = mask.detach().contiguous()
    assert mask.shape == (N, Cin, H, W), (mask.shape, g.shape)
    dx = torch.empty((N, Cin, H, W), dtype=torch.float32, device=g.device)
    L = _lib.lib()
    nprod = 6 if math == "bf16x6" else 3
    ws = _lib.workspace(L.tlod_conv_fwd_bs_workspace_bytes(N, Cout, H, W, Cin, 3, nprod), g.device,
                        "conv")
    _timed("dgrad", (N, Cin, H, W, Cout, 3), lambda: _lib.check(
        L.tlod_conv_dgrad_bs_mask_f32(_lib.ptr(g), _lib.ptr(wp), _lib.ptr(mask), _lib.ptr(dx), N,
                                      Cout, H, W, Cin, nprod, _lib.ptr(ws), ws.numel(),
                                      _lib.stream_of(g)), "conv_dgrad_bs_mask"), math)
    # the tag names the mask and this exact buffer state: autograd may sum another
    # consumer's gradient into dx in place, which bumps _version and voids the tag
    dx._tlod_relu_masked = (mask.data_ptr(), dx.data_ptr(), dx._version)
    STATS["masked_dgrad"] += 1
    return dx


def wgrad_math():
    """Arithmetic of the 3x3 weight gradients (env TLOD_WGRAD_MATH, default: the
    TLOD_CONV_MATH choice): "bf16x6" / "bf16x3" run tlod_conv_wgrad_bs_f32 (split-bf16,
    same slab reduction), "f32" the f32-input MFMA kernel."""
    m = _lib.env("TLOD_WGRAD_MATH") or conv_math()
    if m not in MATHS:
        raise ValueError(f"TLOD_WGRAD_MATH={m!r}: expected one of {MATHS}")
    return m


def conv_wgrad(g, x, KS, out=None, accumulate=False, math=None, db=None, row_scale=None):
    """Weight gradient (into out when given).  db (Cout floats, optional): also the bias
    gradient sum_{n,h,w} g, from the same launch on the split-bf16 path (the f32 path adds
    a reduction pass).  row_scale (Cout, optional): dW[co] scaled by row_scale[co] — in the
    split-bf16 path's reduce (tlod_conv_wgrad_bs_ex_f32), else a pass over dW."""
    g = g.contiguous()
    x = x.contiguous()
    N, Cout, H, W = g.shape
    Cin = x.shape[1]
    L = _lib.lib()
    dw = out if out is not None else torch.empty((Cout, Cin, KS, KS), dtype=torch.float32,
                                                 device=g.device)
    math = wgrad_math() if math is None else math
    if _bs(KS, math) or _wgrad_1x1_bs(KS, math):
        nprod = 6 if math == "bf16x6" else 3
        ws = _lib.workspace(L.tlod_conv_wgrad_bs_workspace_bytes(N, Cin, H, W, Cout, KS, nprod),
                            g.device, "wgrad")
        rs = row_scale.detach().contiguous() if row_scale is not None else None
        _timed("wgrad", (N, Cin, H, W, Cout, KS), lambda: _lib.check(
            L.tlod_conv_wgrad_bs_ex_f32(_lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db),
                                        int(accumulate), _lib.ptr(rs), N, Cin, H, W, Cout, KS,
                                        nprod, _lib.ptr(ws), ws.numel(), _lib.stream_of(g)),
            "conv_wgrad_bs"), math)
        return dw
    if row_scale is not None:
        assert not accumulate
        dw = conv_wgrad(g, x, KS, out, False, math, db)
        return dw.mul_(row_scale.detach().view(-1, 1, 1, 1))
    if db is not None:
        relu_bwd_bias(g, None, want_db=True, db_out=db)
    ws = _lib.workspace(L.tlod_conv_wgrad_workspace_bytes(N, Cin, H, W, Cout, KS), g.device, "wgrad")
    _timed("wgrad", (N, Cin, H, W, Cout, KS), lambda: _lib.check(
        L.tlod_conv_wgrad_f32(_lib.ptr(g), _lib.ptr(x), _lib.ptr(dw), int(accumulate), N, Cin, H, W,
                              Cout, KS, _lib.ptr(ws), ws.numel(), _lib.stream_of(g)), "conv_wgrad"))
    return dw


def relu_bwd_bias(dy, y=None, want_db=True, db_out=None):
    """g = dy * (y > 0) (y None: g = dy); db = sum_{n,h,w} g (into db_out when given)."""
    dy = dy.contiguous()
    N, C, H, W = dy.shape
    g = torch.empty_like(dy) if y is not None else dy
    db = None
    if want_db:
        db = db_out if db_out is not None else torch.empty(C, dtype=torch.float32,
                                                           device=dy.device)
    _lib.check(_lib.lib().tlod_relu_bwd_bias_f32(_lib.ptr(dy), _lib.ptr(y.contiguous() if y is not None else None),
                                                 _lib.ptr(g), _lib.ptr(db), N, C, H * W,
                                                 _lib.stream_of(dy)), "relu_bwd_bias")
    return g, db


_FUSE_RELU = os.environ.get("TLOD_FUSE_RELU", "1") != "0"


def _relu_out(x):
    """x is the ReLU output of a ConvFunction (its ReLU backward can run in the next conv's
    dgrad epilogue; TLOD_FUSE_RELU=0 disables that)."""
    return _FUSE_RELU and getattr(x, "_tlod_relu_out", False)


def _grad_relu(ctx, dy, y, need_b, need_w, bias):
    """(g, db, db_via_wgrad) for a fused-ReLU conv's backward: g = dy * (y > 0).  When dy is
    the next conv's dgrad already masked by y (conv_dgrad(mask=y), tagged) — and not a sum of
    several consumers' gradients (a new tensor, or the tagged one added to in place: its
    _version moved) — the ReLU backward pass is skipped and the bias gradient comes from
    this conv's wgrad launch."""
    if (y is not None and need_w and
            getattr(dy, "_tlod_relu_masked", None) == (y.data_ptr(), dy.data_ptr(), dy._version)):
        STATS["relu_bwd_skipped"] += 1
        db = None
        if need_b:
            db = grad_out(bias)
            if db is None:
                db = torch.empty(dy.shape[1], dtype=torch.float32, device=dy.device)
        return dy, db, True
    g, db = relu_bwd_bias(dy, y, want_db=need_b, db_out=grad_out(bias) if need_b else None)
    return g, db, False


class ConvFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu, tap=None):
        y = conv_fwd(x, weight, bias, relu)
        if tap is not None:  # test instrumentation (Conv2d.act_tap): the activation
            tap.append(y.detach().clone())
        ctx.relu = bool(relu)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)  # gradient slots (tlod.grads)
        ctx.mask_in = _relu_out(x)
        ctx.save_for_backward(x, weight, y if relu else None)
        if relu:
            y._tlod_relu_out = True
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        need_x, need_w, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], \
            ctx.has_bias and ctx.needs_input_grad[2]
        g, db, db_w = _grad_relu(ctx, dy, y if ctx.relu else None, need_b, need_w, ctx.params[1])
        dx = conv_dgrad(g, weight, mask=x if ctx.mask_in else None) if need_x else None
        dw = conv_wgrad(g, x, weight.shape[2], out=grad_out(ctx.params[0]),
                        db=db if db_w else None) if need_w else None
        return dx, dw, db, None, None


def relu_bwd_ex(dy, y=None, scale=None, want_raw=False):
    """g0 = dy * (y > 0) (y None: dy); returns (g0 * scale, g0 or None)."""
    dy = dy.contiguous()
    N, C, H, W = dy.shape
    g = torch.empty_like(dy)
    raw = torch.empty_like(dy) if want_raw else None
    _lib.check(_lib.lib().tlod_relu_bwd_ex_f32(
        _lib.ptr(dy), _lib.ptr(y.contiguous() if y is not None else None),
        _lib.ptr(scale.detach().contiguous() if scale is not None else None), _lib.ptr(g),
        _lib.ptr(raw), None, N, C, H * W, _lib.stream_of(dy)), "relu_bwd_ex")
    return g, raw


class ShortcutLink:
    """Hands an identity bottleneck's shortcut gradient from its conv3's backward (which runs
    first) to its conv1's backward, whose input is the same tensor: conv1's dgrad adds it in
    the epilogue before the previous block's ReLU mask (tlod_conv1x1_gemm_bs_ex_f32), instead
    of autograd summing the two gradients and the previous block running a ReLU-backward pass
    over the sum.  The RoI head's downsample blocks use it the same way for the downsample
    conv's input gradient (LinearActFunction role 4); `consumed` marks that conv1's backward
    has run, so a role-4 backward scheduled after it keeps its gradient for autograd."""

    def __init__(self):
        self.g = None
        self.consumed = False


class ConvBNFunction(torch.autograd.Function):
    """Bias-free conv + frozen BatchNorm (per-channel scale/shift) (+ residual) (+ ReLU), the
    ResNet bottleneck's conv->bn(->add)->relu (lib/DAF/resnet.py:80-99) in one kernel.
    link (a ShortcutLink) with role 3: this conv's residual is its block's input and its
    gradient goes to the link; role 1: this conv reads the block's input and adds the link's
    gradient to its own input gradient."""

    @staticmethod
    def forward(ctx, x, weight, scale, shift, residual, relu, link=None, role=0):
        y = conv_fwd(x, weight, shift, relu, scale=scale, residual=residual)
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.wparam = weight
        ctx.mask_in = _relu_out(x)
        ctx.link, ctx.role = link, role
        ctx.save_for_backward(x, weight, scale, y if relu else None)
        if relu:
            y._tlod_relu_out = True
        return y

    @staticmethod
    def backward(ctx, dy):
        dx, dw, g_res = ConvBNFunction._backward(ctx, dy)
        if ctx.role == 3 and ctx.link is not None and g_res is not None:
            ctx.link.g, g_res = g_res, None  # to conv1's backward (ShortcutLink)
        return (dx, dw, None, None, g_res, None, None, None)[:len(ctx.needs_input_grad)]

    @staticmethod
    def _backward(ctx, dy):
        x, weight, scale, y = ctx.saved_tensors
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_res = ctx.has_res and ctx.needs_input_grad[4]
        mask = x if ctx.mask_in else None
        res = None
        if ctx.role == 1 and ctx.link is not None:
            res, ctx.link.g = ctx.link.g, None
        if (ctx.relu and y is not None and
                getattr(dy, "_tlod_relu_masked", None) == (y.data_ptr(), dy.data_ptr(), dy._version)):
            # dy is the next conv's dgrad, already masked by this ReLU (a bottleneck's 3x3 conv2
            # masks conv1's gradient): the BN scale g = dy * scale folds into the dgrad weight
            # (W * scale per output channel) and the weight gradient's rows — no pass over dy
            STATS["relu_bwd_skipped"] += 1
            dx = (conv_dgrad(dy, weight, mask=mask, residual=res, wscale=scale)
                  if need_x else None)
            dw = (conv_wgrad(dy, x, weight.shape[2], out=grad_out(ctx.wparam), row_scale=scale)
                  if need_w else None)
            return dx, dw, dy if need_res else None
        g, g_raw = relu_bwd_ex(dy, y if ctx.relu else None, scale, want_raw=need_res)
        dx = conv_dgrad(g, weight, mask=mask, residual=res) if need_x else None
        dw = conv_wgrad(g, x, weight.shape[2], out=grad_out(ctx.wparam)) if need_w else None
        return dx, dw, g_raw


def maxpool2x2(x):
    """nn.MaxPool2d(2, 2) (floor mode) forward in libtlod (tlod_maxpool2x2_f32)."""
    x = x.contiguous()
    N, C, H, W = x.shape
    y = torch.empty((N, C, H // 2, W // 2), dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().tlod_maxpool2x2_f32(_lib.ptr(x), N, C, H, W, _lib.ptr(y),
                                              _lib.stream_of(x)), "maxpool2x2")
    return y


def maxpool_relu_bwd(dp, y, want_db=True, db_out=None):
    """Gradient through max_pool2d(2, 2) and the ReLU whose output y the pool read:
    g = dp routed to each window's argmax where y > 0; db = sum g (into db_out if given)."""
    dp = dp.contiguous()
    N, C, H, W = y.shape
    g = torch.empty_like(y)
    db = None
    if want_db:
        db = db_out if db_out is not None else torch.empty(C, dtype=torch.float32,
                                                           device=y.device)
    _lib.check(_lib.lib().tlod_maxpool2x2_relu_bwd_f32(_lib.ptr(dp), _lib.ptr(y), N, C, H, W,
                                                       _lib.ptr(g), _lib.ptr(db),
                                                       _lib.stream_of(y)), "maxpool_relu_bwd")
    return g, db


def conv_fwd_pool(x, weight, bias, math=None):
    """max_pool2d(relu(conv(x) + bias), 2, 2) with the pooling in the conv epilogue (split-bf16
    3x3, tlod_conv_fwd_bs_pool_f32): the full-resolution map is never written.  Forward only
    (frozen layers); other maths pool in a separate kernel."""
    _check(x, weight)
    x = x.contiguous()
    N, Cin, H, W = x.shape
    Cout, _, KS, _ = weight.shape
    math = conv_math() if math is None else math
    if not _bs(KS, math):
        return maxpool2x2(conv_fwd(x, weight, bias, True, math=math))
    y = torch.empty((N, Cout, H // 2, W // 2), dtype=torch.float32, device=x.device)
    b = bias.detach().contiguous() if bias is not None else None
    nprod = 6 if math == "bf16x6" else 3
    wp = pack_bs(weight, False)
    _timed("fwd", (N, Cin, H, W, Cout, KS), lambda: _lib.check(
        _lib.lib().tlod_conv_fwd_bs_pool_f32(_lib.ptr(x), _lib.ptr(wp), None, _lib.ptr(b),
                                             _lib.ptr(y), N, Cin, H, W, Cout, KS, 1, nprod,
                                             _lib.stream_of(x)), "conv_fwd_bs_pool"), math)
    return y


class ConvPoolFunction(torch.autograd.Function):
    """conv + bias + ReLU + max_pool2d(2, 2) as one autograd node: the backward routes the
    pooled gradient through the recomputed argmax and the ReLU mask in one kernel
    (tlod_maxpool2x2_relu_bwd_f32) — no index tensor, no full-size pool gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, tap=None):
        y = conv_fwd(x, weight, bias, True)
        if tap is not None:  # test instrumentation: the pre-pool activation
            tap.append(y.detach().clone())
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.mask_in = _relu_out(x)
        ctx.save_for_backward(x, weight, y)
        return maxpool2x2(y)

    @staticmethod
    def backward(ctx, dp):
        x, weight, y = ctx.saved_tensors
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        g, db = maxpool_relu_bwd(dp, y, want_db=need_b,
                                 db_out=grad_out(ctx.params[1]) if need_b else None)
        dx = conv_dgrad(g, weight, mask=x if ctx.mask_in else None) if need_x else None
        dw = conv_wgrad(g, x, weight.shape[2], out=grad_out(ctx.params[0])) if need_w else None
        return dx, dw, db, None


class Conv1x1SmallFunction(torch.autograd.Function):
    """1x1 conv with 1 <= Cout <= 4 (no ReLU): _ImageDA.Conv2 (512 -> 2, lib/DAF/DA.py:36-50)
    on the streaming kernels of csrc/conv_small.hip (tlod_conv1x1_small_{fwd,dgrad,wgrad}_f32)
    instead of F.linear over a channels-last copy.  The weight gradient is written into its
    arena slot when one is free (tlod.grads)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _lib.require_cuda(x, weight)
        x = x.contiguous()
        N, Cin, H, W = x.shape
        Cout = weight.shape[0]
        w = weight.detach().reshape(Cout, Cin).contiguous()
        b = bias.detach().contiguous() if bias is not None else None
        y = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib().tlod_conv1x1_small_fwd_f32(
            _lib.ptr(x), N, Cin, H, W, _lib.ptr(w), _lib.ptr(b), Cout, _lib.ptr(y),
            _lib.stream_of(x)), "conv1x1_small_fwd")
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        weight, bias = ctx.params
        dy = dy.contiguous()
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        L = _lib.lib()
        st = _lib.stream_of(dy)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _lib.check(L.tlod_conv1x1_small_dgrad_f32(_lib.ptr(dy), N, Cout, H, W, _lib.ptr(w),
                                                      Cin, _lib.ptr(dx), st), "conv1x1_small_dgrad")
        need_b = bias is not None and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or need_b:
            dw = grad_out(weight) if ctx.needs_input_grad[1] else None
            if dw is None:
                dw = torch.empty_like(weight)
            if need_b:
                db = grad_out(bias)
                if db is None:
                    db = torch.empty_like(bias)
            ws = _lib.workspace(L.tlod_conv1x1_small_wgrad_workspace_bytes(N, Cin, H, W, Cout),
                                dy.device, "conv1x1_small")
            _lib.check(L.tlod_conv1x1_small_wgrad_f32(
                _lib.ptr(dy), _lib.ptr(x), N, Cin, H, W, Cout, _lib.ptr(dw), _lib.ptr(db),
                _lib.ptr(ws), ws.numel(), st), "conv1x1_small_wgrad")
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db


class Conv2d(nn.Conv2d):
    """nn.Conv2d-compatible (stride 1, padding k//2) with the libtlod kernels; optional
    fused ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=None, bias=True,
                 relu=False):
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        padding = k // 2 if padding is None else padding
        super().__init__(in_channels, out_channels, k, stride=stride, padding=padding, bias=bias)
        if stride != 1 or padding != k // 2 or k not in (1, 3):
            raise NotImplementedError("tlod.Conv2d: stride 1, 'same' padding, 1x1/3x3 only")
        self.relu = relu
        self.pool = False  # set by the VGG16 builder: max_pool2d(2, 2) of the ReLU output
        self.act_tap = None  # tests: a list receiving each forward's (pre-pool) activation

    def forward(self, x):
        if self.pool:
            assert self.relu
            needs_grad = torch.is_grad_enabled() and (
                x.requires_grad or self.weight.requires_grad
                or (self.bias is not None and self.bias.requires_grad))
            if not needs_grad:
                return conv_fwd_pool(x, self.weight, self.bias)
            return ConvPoolFunction.apply(x, self.weight, self.bias, self.act_tap)
        if self.out_channels <= 4 and self.kernel_size[0] == 1 and not self.relu:
            return Conv1x1SmallFunction.apply(x, self.weight, self.bias)
        if self.out_channels % 4:
            # GEMM-library path for other odd-width 1x1 heads
            assert self.kernel_size[0] == 1
            y = F.linear(x.permute(0, 2, 3, 1), self.weight.view(self.out_channels, -1), self.bias)
            y = y.permute(0, 3, 1, 2).contiguous()
            return F.relu(y) if self.relu else y
        return ConvFunction.apply(x, self.weight, self.bias, self.relu, self.act_tap)

    def extra_repr(self):
        return super().extra_repr() + (", relu=True" if self.relu else "") + \
            (", maxpool2x2" if self.pool else "")


def vgg_init_(conv):
    """torchvision 0.2.1 VGG init (reference requirements.txt:1): N(0, sqrt(2/(k*k*out))), bias 0."""
    n = conv.kernel_size[0] * conv.kernel_size[1] * conv.out_channels
    conv.weight.data.normal_(0, math.sqrt(2.0 / n))
    if conv.bias is not None:
        conv.bias.data.zero_()
