"""Fully connected layers on libtlod's split-bf16 GEMM (tlod_gemm_bs_f32).

``Linear`` is a drop-in for the ``nn.Linear`` modules of the detection head
(RCNN_top = torchvision vgg16().classifier[:-1]: fc6 25088->4096, fc7 4096->4096,
lib/DAF/vgg16.py:67-71) and of the DA instance discriminator (lib/DAF/DA.py:53-73): same
parameters, same state_dict keys, same init.  Forward, input gradient and weight gradient
each run as one GEMM in libtlod (operands split exactly into bf16 planes on the fly, f32
accumulation: f32-level error, tests/test_linear_gpu.py); the bias gradient is a column
sum.  Layers narrower than one 256-wide tile (the 9-way class / 36-way box heads, the
1-way DA classifier) stay on nn.Linear, where a 256x256 tile would be mostly padding.
"""

import torch
import torch.nn as nn

from . import _lib
from .grads import grad_out

MATHS = ("bf16x6", "bf16x3")


def linear_math():
    """TLOD_LINEAR_MATH: "bf16x6" (default, f32-level error), "bf16x3" (~5e-6), or "f32"
    (nn.Linear's GEMM library path, for A/B comparison)."""
    m = _lib.env("TLOD_LINEAR_MATH", "bf16x6")
    if m not in MATHS + ("f32",):
        raise ValueError(f"TLOD_LINEAR_MATH={m!r}")
    return m


def gemm(a, b, M, N, K, a_kcontig, b_kcontig, bias=None, math="bf16x6", out=None,
         residual=None, relu=False):
    """c[M][N] = act(sum_k A(m,k) B(n,k) (+ bias[n]) (+ residual[m][n])) — see include/tlod.h
    tlod_gemm_bs_f32 / tlod_gemm_bs_ex_f32.  ``out``: a contiguous (M, N) float32 tensor to
    write into."""
    _lib.require_cuda(a, b)
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("tlod gemm computes in fp32 (the reference's dtype)")
    a, b = a.contiguous(), b.contiguous()
    nprod = 6 if math == "bf16x6" else 3
    L = _lib.lib()
    c = torch.empty((M, N), dtype=torch.float32, device=a.device) if out is None else out
    assert c.is_contiguous() and c.numel() == M * N
    ws = _lib.workspace(L.tlod_gemm_bs_workspace_bytes(M, N, K, a_kcontig, b_kcontig, nprod),
                        a.device, "gemm")
    bias = bias.detach().contiguous() if bias is not None else None
    from .conv import _timed  # bench.py's launch timing (tlod.conv.PROFILE), shape (M, N, K)
    if residual is None and not relu:
        _timed("gemm", (M, N, K), lambda: _lib.check(
            L.tlod_gemm_bs_f32(_lib.ptr(a), _lib.ptr(b), _lib.ptr(bias), _lib.ptr(c), M, N, K,
                               int(a_kcontig), int(b_kcontig), nprod, _lib.ptr(ws), ws.numel(),
                               _lib.stream_of(a)), "gemm_bs"), math)
        return c
    if residual is not None:
        residual = residual.detach().contiguous()
        assert residual.shape == (M, N) and residual.dtype == torch.float32
    _timed("gemm", (M, N, K), lambda: _lib.check(
        L.tlod_gemm_bs_ex_f32(_lib.ptr(a), _lib.ptr(b), _lib.ptr(bias), _lib.ptr(residual),
                              int(relu), _lib.ptr(c), M, N, K, int(a_kcontig), int(b_kcontig),
                              nprod, _lib.ptr(ws), ws.numel(), _lib.stream_of(a)), "gemm_bs_ex"),
        math)
    return c


class LinearFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, math):
        R, I = x.shape
        O = weight.shape[0]
        y = gemm(x, weight.detach(), R, O, I, 1, 1, bias, math)          # x W^T (+ b)
        ctx.math = math
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)  # gradient slots (tlod.grads)
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        R, I = x.shape
        O = weight.shape[0]
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dy, weight.detach(), R, I, O, 1, 0, None, ctx.math)  # dy W
        if ctx.needs_input_grad[1]:
            dw = gemm(dy, x, O, I, R, 0, 0, None, ctx.math,                # dy^T x
                      out=grad_out(ctx.params[0]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            slot = grad_out(ctx.params[1])
            db = dy.sum(0) if slot is None else torch.sum(dy, 0, out=slot)
        return dx, dw, db, None


def gemm_mask(a, b, M, N, K, a_kcontig, b_kcontig, mask, residual=None, math="bf16x6"):
    """c = (A.B (+ residual)) * (mask > 0): an input gradient through the ReLU whose output
    (mask) the GEMM read, with an identity shortcut's gradient added first
    (tlod_gemm_bs_mask_f32).  The result is tagged for LinearActFunction's backward."""
    a, b = a.contiguous(), b.contiguous()
    mask = mask.detach().contiguous()
    nprod = 6 if math == "bf16x6" else 3
    L = _lib.lib()
    c = torch.empty((M, N), dtype=torch.float32, device=a.device)
    ws = _lib.workspace(L.tlod_gemm_bs_workspace_bytes(M, N, K, a_kcontig, b_kcontig, nprod),
                        a.device, "gemm")
    if residual is not None:
        residual = residual.detach().contiguous()
        assert residual.shape == (M, N)
    from .conv import _timed
    _timed("gemm", (M, N, K), lambda: _lib.check(
        L.tlod_gemm_bs_mask_f32(_lib.ptr(a), _lib.ptr(b), _lib.ptr(residual), _lib.ptr(mask),
                                _lib.ptr(c), M, N, K, int(a_kcontig), int(b_kcontig), nprod,
                                _lib.ptr(ws), ws.numel(), _lib.stream_of(a)), "gemm_bs_mask"),
        math)
    c._tlod_relu_masked = (mask.data_ptr(), c.data_ptr(), c._version)
    STATS["masked_dgrad"] += 1
    return c


def gemm_nhwc3(mode, a, b, R, H, W, C, O, bias=None, residual=None, mask=None, relu=False,
               math="bf16x6", out=None):
    """The RoI head's 3x3 conv as an implicit GEMM over channels-last (R*H*W, .) rows
    (tlod_gemm_nhwc3_bs_f32): mode 0 forward (a = x, b = the (O, 9C) weight rows), 1 input
    gradient (a = dy, b = the (9O, C) flipped weight; mask: the input's ReLU output, the
    result tagged as masked), 2 weight gradient (a = dy, b = x) -> (O, 9C)."""
    a, b = a.contiguous(), b.contiguous()
    nprod = 6 if math == "bf16x6" else 3
    L = _lib.lib()
    rows = R * H * W
    shape = {0: (rows, O), 1: (rows, C), 2: (O, 9 * C)}[mode]
    c = torch.empty(shape, dtype=torch.float32, device=a.device) if out is None else out
    assert c.is_contiguous() and c.numel() == shape[0] * shape[1]
    ws = _lib.workspace(L.tlod_gemm_nhwc3_bs_workspace_bytes(mode, R, H, W, C, O, nprod),
                        a.device, "gemm")
    bias = bias.detach().contiguous() if bias is not None else None
    residual = residual.detach().contiguous() if residual is not None else None
    mask = mask.detach().contiguous() if mask is not None else None
    from .conv import _timed
    mnk = {0: (rows, O, 9 * C), 1: (rows, C, 9 * O), 2: (O, 9 * C, rows)}[mode]
    _timed("gemm", mnk, lambda: _lib.check(
        L.tlod_gemm_nhwc3_bs_f32(mode, _lib.ptr(a), _lib.ptr(b), _lib.ptr(bias),
                                 _lib.ptr(residual), _lib.ptr(mask), int(relu), _lib.ptr(c), R, H,
                                 W, C, O, nprod, _lib.ptr(ws), ws.numel(), _lib.stream_of(a)),
        "gemm_nhwc3_bs"), math)
    if mask is not None:
        c._tlod_relu_masked = (mask.data_ptr(), c.data_ptr(), c._version)
        STATS["masked_dgrad"] += 1
    return c


STATS = {"masked_dgrad": 0, "relu_bwd_skipped": 0}  # fused ReLU-backward counters (tests)


class LinearActFunction(torch.autograd.Function):
    """y = act(x W^T + bias + residual) in one GEMM launch (the ResNet RoI head's bottleneck
    convs as GEMMs with the folded BN shift as the bias, lib/DAF/resnet.py Bottleneck:
    out = relu(bn3(conv3(...)) + residual)).  Backward: g = dy * (y > 0), then the GEMMs of
    LinearFunction; the residual's gradient is g.
    relu_in: x is a ReLU output — the input gradient is masked in the GEMM epilogue
    (gemm_mask) and tagged, so that layer's backward skips its own mask pass (a gradient that
    arrives tagged for this y is already g).  link (a tlod.conv.ShortcutLink) / role: an
    identity bottleneck's conv3 (role 3) hands its residual gradient g to conv1 (role 1),
    whose input gradient adds it in the same epilogue — no autograd sum of the two; a
    downsample block's shortcut conv (role 4) hands conv1 its input gradient the same way.
    wsrc / wscale (a conv weight (O, C, kh, kw) and a per-output scale): `weight` is the GEMM
    form of wsrc * wscale (rows (kh, kw, c) for 3x3), computed by the caller without autograd;
    the backward writes d wsrc = (dy^T x in the GEMM form) * wscale, re-laid out, straight
    into wsrc's gradient slot (one pass) instead of autograd's mul, permute copy and the
    arena's copy of the result.
    nhwc3 = (R, H, W) (round 6): x is not the im2col matrix of a 3x3 conv but its channels-last
    input map rows (R*H*W, C), and weight the (O, 9C) rows — the three GEMMs run as implicit
    GEMMs over the map (gemm_nhwc3: no im2col / col2im passes, no (R*H*W, 9C) tensor saved)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, relu, math, relu_in=False, link=None, role=0,
                wsrc=None, wscale=None, mean_hw=None, nhwc3=None):
        R, I = x.shape
        O = weight.shape[0]
        ctx.nhwc3 = nhwc3
        if nhwc3 is not None:
            y = gemm_nhwc3(0, x, weight.detach(), *nhwc3, I, O, bias=bias, residual=residual,
                           relu=relu, math=math)
        else:
            y = gemm(x, weight.detach(), R, O, I, 1, 1, bias, math, residual=residual, relu=relu)
        ctx.mean_hw = mean_hw
        ctx.math, ctx.relu = math, relu
        ctx.has_bias, ctx.has_res = bias is not None, residual is not None
        ctx.params = (weight, bias)
        ctx.relu_in, ctx.link, ctx.role = bool(relu_in), link, role
        ctx.wsrc, ctx.wscale = wsrc, wscale
        ctx.save_for_backward(x, weight, y if relu else None)
        if mean_hw is not None:
            # the ResNet head's fc7 = y.view(R, H, W, O).mean(2).mean(1) (resnet.py:286-288)
            # taken here, so the backward builds its gradient straight from the (R, O) mean
            # gradient (no (R*H*W, O) broadcast materialised by a view's backward)
            Rr, H, W = mean_hw
            return y.view(Rr, H, W, O).mean(2).mean(1)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        R, I = x.shape
        O = weight.shape[0]
        if ctx.mean_hw is not None:  # dy: (Rr, O), the two means' backward is (dy / H) / W
            Rr, H, W = ctx.mean_hw
            gb = ((dy / H) / W)[:, None, :].expand(Rr, H * W, O)
            if ctx.relu:
                g = torch.where(y.view(Rr, H * W, O) > 0, gb,
                                torch.zeros((), dtype=dy.dtype, device=dy.device)).view(R, O)
            else:
                g = gb.reshape(R, O)
        elif ctx.relu and getattr(dy, "_tlod_relu_masked", None) == (y.data_ptr(), dy.data_ptr(),
                                                                     dy._version):
            g = dy  # masked by the consumer's input-gradient epilogue
            STATS["relu_bwd_skipped"] += 1
        elif ctx.relu:  # (one pass: dy may be a broadcast view, e.g. the head's mean backward)
            g = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
        else:
            g = dy.contiguous()
        res = None
        if ctx.role == 1 and ctx.link is not None:
            res, ctx.link.g = ctx.link.g, None
            ctx.link.consumed = True  # a role-4 backward running later returns its own dx
        dx = dw = db = None
        n3 = ctx.nhwc3
        if n3 is not None:  # implicit 3x3 GEMMs over the map (I = C channels here)
            def wgrad(out=None):
                return gemm_nhwc3(2, g, x, *n3, I, O, math=ctx.math, out=out)
            if ctx.needs_input_grad[0]:
                with torch.no_grad():  # row (t, o) = weight row o at tap 8 - t
                    wd = weight.detach().view(O, 9, I).flip(1).transpose(0, 1).reshape(9 * O, I)
                dx = gemm_nhwc3(1, g, wd, *n3, I, O, residual=res,
                                mask=x if ctx.relu_in else None, math=ctx.math)
        else:
            def wgrad(out=None):
                return gemm(g, x, O, I, R, 0, 0, None, ctx.math, out=out)
            if ctx.needs_input_grad[0]:
                if ctx.relu_in:
                    dx = gemm_mask(g, weight.detach(), R, I, O, 1, 0, x, res, ctx.math)
                else:
                    dx = gemm(g, weight.detach(), R, I, O, 1, 0, None, ctx.math, residual=res)
        if ctx.needs_input_grad[1]:
            dw = wgrad(out=grad_out(ctx.params[0]))
        if (dx is not None and ctx.role == 4 and ctx.link is not None
                and not getattr(ctx.link, "consumed", False)):
            ctx.link.g, dx = dx, None  # to conv1's input-gradient GEMM (role 1)
        dsrc = None
        if ctx.wsrc is not None and ctx.needs_input_grad[9]:
            w = ctx.wsrc
            dwg = wgrad()  # (O, I) in the GEMM layout (3x3: (O, 9C))
            slot = grad_out(w)
            dsrc = slot if slot is not None else torch.empty_like(w)
            sc = ctx.wscale.detach()
            if w.shape[2] == 1:
                torch.mul(dwg, sc[:, None], out=dsrc.view(O, -1))
            else:  # rows (kh, kw, c) -> (c, kh, kw)
                kh, kw = w.shape[2], w.shape[3]
                torch.mul(dwg.view(O, kh, kw, -1).permute(0, 3, 1, 2), sc.view(-1, 1, 1, 1),
                          out=dsrc)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            slot = grad_out(ctx.params[1])
            db = g.sum(0) if slot is None else torch.sum(g, 0, out=slot)
        dres = g if ctx.has_res and ctx.needs_input_grad[3] else None
        if dres is not None and ctx.role == 3 and ctx.link is not None:
            ctx.link.g, dres = dres, None  # to conv1's backward
        return dx, dw, db, dres, None, None, None, None, None, dsrc, None, None, None


class Linear(nn.Linear):
    """nn.Linear with the libtlod GEMM (2-D input [rows, in_features])."""

    def forward(self, x):
        m = linear_math()
        if m == "f32" or x.dim() != 2:
            return super().forward(x)
        return LinearFunction.apply(x, self.weight, self.bias, m)


def fused_act():
    """TLOD_FUSED_ACT (default 1): ReLU + dropout after the head's Linear layers as one
    libtlod pass each way (tlod_relu_dropout_f32); 0 = nn.ReLU + nn.Dropout."""
    return _lib.env("TLOD_FUSED_ACT", "1") != "0"


class ReluDropoutFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, p, seed):
        _lib.require_cuda(y)
        y = y.contiguous()
        out = torch.empty_like(y)
        _lib.check(_lib.lib().tlod_relu_dropout_f32(_lib.ptr(y), _lib.ptr(out), y.numel(), float(p),
                                                    seed, _lib.stream_of(y)), "relu_dropout")
        ctx.p = float(p)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dout):
        (out,) = ctx.saved_tensors
        dout = dout.contiguous()
        g = torch.empty_like(out)
        _lib.check(_lib.lib().tlod_relu_dropout_bwd_f32(_lib.ptr(dout), _lib.ptr(out), _lib.ptr(g),
                                                        out.numel(), ctx.p, _lib.stream_of(out)),
                   "relu_dropout_bwd")
        return g, None, None


def relu_dropout(y, dropout, tap=None):
    """dropout(relu(y)) with the nn.Dropout module's p and training mode (its RNG stream is
    libtlod's counter-based one, seeded from torch's CPU generator: no device sync; no draw
    at all when p == 0 or in eval mode, so the CPU generator's stream is left alone)."""
    p = float(dropout.p) if dropout.training else 0.0
    if not fused_act():
        return dropout(torch.relu(y))
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0.0 else 0
    out = ReluDropoutFunction.apply(y, p, seed)
    if tap is not None:  # test instrumentation (Linear.act_tap): the activation
        tap.append(out.detach().clone())
    return out


class FcTop(nn.Sequential):
    """nn.Sequential(Linear, ReLU, Dropout, Linear, ReLU, Dropout) — the VGG16 RCNN_top,
    same modules and state_dict keys — whose Linear -> ReLU -> Dropout triples run as the
    split-bf16 GEMM (bias in its epilogue) plus one fused ReLU + dropout pass."""

    def forward(self, x):
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            if (i + 2 < len(mods) and isinstance(m, nn.Linear) and isinstance(mods[i + 1], nn.ReLU)
                    and isinstance(mods[i + 2], nn.Dropout)):
                x = relu_dropout(m(x), mods[i + 2], getattr(m, "act_tap", None))
                i += 3
            else:
                x = m(x)
                i += 1
        return x
