"""ResNet101 backbone and head for the DAF/MAF/ATF detectors (lib/DAF/resnet.py:57-288).

Same modules and state_dict keys as the reference (``RCNN_base`` = Sequential(conv1, bn1,
relu, maxpool, layer1, layer2, layer3), ``RCNN_top`` = Sequential(layer4); Bottleneck
conv1/bn1/conv2/bn2/conv3/bn3/downsample), the caffe-style stride on the bottleneck's 1x1
conv1 (:71), maxpool ceil_mode (:113), frozen conv1/bn1/layer1 and every BatchNorm frozen
in eval mode (:249-284).  Execution:

  * every BatchNorm is frozen and in eval mode, i.e. a per-channel affine, folded into
    the producing conv's epilogue (tlod_conv_fwd_ex_f32: conv * scale + shift
    (+ residual) (+ ReLU)) — one kernel per conv, no separate BN / add / ReLU passes;
  * stride-2 1x1 convs run as the stride-1 conv of x[:, :, ::2, ::2] (tlod_subsample2_f32;
    conv1 and the downsample share the subsampled tensor);
  * the stem (7x7/2 conv + bn1 + ReLU, frozen) is tlod_stem_conv7x7s2_f32;
  * the RoI head (layer4 on R x 1024 x 7x7 -> 4x4 maps) runs channels-last: 1x1 convs
    are plain GEMMs and the 3x3 convs GEMMs over a 9-tap gather, on libtlod's split-bf16
    GEMM (tlod.linear; TLOD_LINEAR_MATH=f32: hipBLASLt through torch.addmm) — 4x4 maps
    would fill 16 of the 256 pixel slots of a conv tile.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..config import cfg
from .. import conv as conv_mod
from ..conv import ConvBNFunction, ShortcutLink
from ..linear import LinearActFunction, linear_math


def fold_bn(bn):
    """Frozen eval-mode BatchNorm as y = x * scale + shift (per channel).  Cached on the
    module and recomputed only when one of its four tensors changes: a different tensor object
    (reassignment, load_state_dict(assign=True)), new storage under the same object
    (module.to() / .cuda(): param.data = ...), an in-place write (its version counter) or a
    write that bypasses it (tlod.conv.weights_updated: the data-parallel broadcast).
    The cache holds the four tensors themselves, so a replaced tensor's storage cannot be
    reused at the same address while its fold is cached.  ResNet101 has 104 BatchNorms, i.e.
    400+ small launches per forward otherwise."""
    assert not bn.weight.requires_grad, "tlod ResNet expects frozen BatchNorm (resnet.py:261-267)"
    ts = (bn.weight, bn.bias, bn.running_mean, bn.running_var)
    # (data_ptr / device / dtype: module.to() and .cuda() swap a parameter's storage through
    # param.data = ..., which keeps the object and its version counter)
    vs = tuple((t._version, t.data_ptr(), t.device, t.dtype) for t in ts) + (
        bn.eps, conv_mod._EXTERNAL_WRITES[0])
    c = getattr(bn, "_tlod_fold", None)
    if c is not None and c[1] == vs and all(a is b for a, b in zip(c[0], ts)):
        return c[2], c[3]
    with torch.no_grad():
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        shift = bn.bias - bn.running_mean * scale
    scale, shift = scale.contiguous(), shift.contiguous()
    bn._tlod_fold = (ts, vs, scale, shift)
    return scale, shift


class Subsample2Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _lib.require_cuda(x)
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty((N, C, (H + 1) // 2, (W + 1) // 2), dtype=x.dtype, device=x.device)
        _lib.check(_lib.lib().tlod_subsample2_f32(_lib.ptr(x), N, C, H, W, _lib.ptr(y),
                                                  _lib.stream_of(x)), "subsample2")
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        g = g.contiguous()
        dx = torch.empty((N, C, H, W), dtype=g.dtype, device=g.device)
        _lib.check(_lib.lib().tlod_upsample2_zero_f32(_lib.ptr(g), N, C, H, W, _lib.ptr(dx),
                                                      _lib.stream_of(g)), "upsample2_zero")
        return dx


class Im2col3x3Function(torch.autograd.Function):
    """x (R,H,W,C) channels-last -> (R*H*W, 9*C) taps in (kh, kw, c) order, zero padding 1
    (tlod_im2col3x3_nhwc_f32; backward tlod_col2im3x3_nhwc_f32).  shape (R, H, W): x is the
    same map as (R*H*W, C) rows (the head's GEMM outputs, no autograd view in between);
    relu_in: x is a ReLU output, so the backward applies its mask in the col2im pass
    (tlod_col2im3x3_nhwc_mask_f32) and tags the gradient for LinearActFunction."""

    @staticmethod
    def forward(ctx, x, shape=None, relu_in=False):
        _lib.require_cuda(x)
        x = x.contiguous()
        R, H, W = shape if shape is not None else x.shape[:3]
        C = x.shape[-1]
        col = torch.empty((R * H * W, 9 * C), dtype=x.dtype, device=x.device)
        _lib.check(_lib.lib().tlod_im2col3x3_nhwc_f32(_lib.ptr(x), R, H, W, C, _lib.ptr(col),
                                                      _lib.stream_of(x)), "im2col3x3_nhwc")
        ctx.shape, ctx.in_shape = (R, H, W, C), x.shape
        ctx.save_for_backward(x if relu_in else None)
        return col

    @staticmethod
    def backward(ctx, g):
        R, H, W, C = ctx.shape
        (x,) = ctx.saved_tensors
        g = g.contiguous()
        dx = torch.empty(ctx.in_shape, dtype=g.dtype, device=g.device)
        _lib.check(_lib.lib().tlod_col2im3x3_nhwc_mask_f32(
            _lib.ptr(g), R, H, W, C, _lib.ptr(x), _lib.ptr(dx), _lib.stream_of(g)),
            "col2im3x3_nhwc")
        if x is not None:
            dx._tlod_relu_masked = (x.data_ptr(), dx.data_ptr(), dx._version)
        return dx, None, None


def im2col3x3_nhwc(x, shape=None, relu_in=False):
    """x: (R, H, W, C), or (R*H*W, C) rows with shape = (R, H, W)."""
    if x.shape[-1] % 4 == 0:
        return Im2col3x3Function.apply(x, shape, relu_in)
    if shape is not None:
        x = x.view(*shape, x.shape[-1])
    R, H, W, P = x.shape  # (unaligned channel counts: the torch composition)
    pad = F.pad(x, (0, 0, 1, 1, 1, 1))
    return torch.cat([pad[:, kh:kh + H, kw:kw + W, :] for kh in range(3) for kw in range(3)],
                     3).reshape(R * H * W, 9 * P)


def conv_bn(x, conv, bn, relu, residual=None, link=None, role=0):
    scale, shift = fold_bn(bn)
    return ConvBNFunction.apply(x, conv.weight, scale, shift, residual, relu, link, role)


def stem(x, conv1, bn1):
    """conv1 7x7/2 + bn1 + ReLU (resnet.py:107-110; frozen: forward only)."""
    _lib.require_cuda(x)
    assert not conv1.weight.requires_grad
    x = x.contiguous()
    N, _, H, W = x.shape
    scale, shift = fold_bn(bn1)
    y = torch.empty((N, 64, (H - 1) // 2 + 1, (W - 1) // 2 + 1), dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib().tlod_stem_conv7x7s2_f32(
        _lib.ptr(x), _lib.ptr(conv1.weight.detach().contiguous()), _lib.ptr(scale),
        _lib.ptr(shift), _lib.ptr(y), N, H, W, 1, _lib.stream_of(x)), "stem_conv")
    return y


class Bottleneck(nn.Module):
    """resnet.py:64-102 (modules for parameters/keys; forward on the fused kernels)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.act_tap = None  # tests: {"r1"|"r2"|"r3": list} receiving each ReLU's mask (NCHW)

    def _tap(self, tag, y, nhwc=False):
        if self.act_tap is not None:
            m = y.detach() > 0
            self.act_tap[tag].append(m.permute(0, 3, 1, 2) if nhwc else m)
        return y

    def forward(self, x):
        xs = Subsample2Function.apply(x) if self.stride == 2 else x
        # identity shortcut: conv1's dgrad takes the shortcut's gradient (ShortcutLink)
        link = ShortcutLink() if self.downsample is None and self.stride == 1 else None
        out = self._tap("r1", conv_bn(xs, self.conv1, self.bn1, relu=True, link=link, role=1))
        out = self._tap("r2", conv_bn(out, self.conv2, self.bn2, relu=True))
        res = (conv_bn(xs, self.downsample[0], self.downsample[1], relu=False)
               if self.downsample is not None else x)
        return self._tap("r3", conv_bn(out, self.conv3, self.bn3, relu=True, residual=res,
                                       link=link, role=3))

    # ---------------------------------------------------------------- RoI head path
    @staticmethod
    def _gemm_bn(xm, conv, bn, relu, residual=None, relu_in=False, link=None, role=0,
                 mean_hw=None, nhwc3=None):
        """xm: (P, Cin) channels-last rows; conv as a GEMM + folded BN (+res) (+ReLU).
        relu_in: xm is a ReLU output (its input gradient is masked in the GEMM epilogue);
        link / role: the identity shortcut's gradient handed from conv3 (role 3) to conv1
        (role 1) — see LinearActFunction.  mean_hw = (R, H, W): return the head's spatial
        mean (R, Cout) instead of the rows (split-bf16 path only; the caller checks).
        nhwc3 = (R, H, W): conv is 3x3 and xm its input map's rows, not the im2col matrix
        (the implicit GEMMs; split-bf16 path only, the caller checks)."""
        scale, shift = fold_bn(bn)
        w = conv.weight
        wm = w.view(w.shape[0], -1) if w.shape[2] == 1 else w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        # BN scale folded into the (small) weight, shift as the GEMM's bias: one GEMM with
        # its bias epilogue instead of GEMM + two passes over the (R*H*W, C) output; the
        # GEMMs (forward, input and weight gradient) on libtlod's split-bf16 GEMM
        m = linear_math()
        if m == "f32":
            y = torch.addmm(shift, xm, (wm * scale[:, None]).t())
            if residual is not None:
                y = y.add_(residual)
            return F.relu(y, inplace=True) if relu else y
        # residual add and ReLU in the GEMM epilogue (tlod_gemm_bs_ex_f32); the folded weight
        # is built outside autograd and the weight gradient written into the conv weight's
        # slot by the GEMM function (wsrc / wscale)
        with torch.no_grad():
            wf = (wm * scale[:, None]).contiguous()
        return LinearActFunction.apply(xm.contiguous(), wf, shift, residual, relu, m, relu_in,
                                       link, role, w, scale, mean_hw, nhwc3)

    def forward_nhwc(self, x, subsampled=False, shape=None, relu_in=False, mean=False):
        """The layer4 RoI head, channels-last.  x: (R, H, W, C), or (R*H*W, C) rows with
        shape = (R, H, W) (a previous block's output, relu_in = True); returns (rows, shape).
        subsampled: x is already the stride-2 subsample (the head entry, HeadEntry).
        mean (the head's last block): when the fused path runs, returns (the spatial mean
        (R, C), None) — fc7 of _head_to_tail — taken inside conv3's GEMM function."""
        if shape is None:
            if self.stride == 2 and not subsampled:
                x = x[:, ::2, ::2, :]
            R, H, W, C = x.shape
            xm = x.reshape(R * H * W, C)
        else:
            assert self.stride == 1 or subsampled
            (R, H, W), xm = shape, x
        fused = linear_math() != "f32" and _lib.env("TLOD_HEAD_FUSE", "1") != "0"
        # identity shortcut: conv1's input gradient takes the shortcut's gradient (conv3's
        # residual gradient, role 3); downsample shortcut: it takes the downsample conv's
        # input gradient (role 4) — either way one GEMM epilogue instead of autograd's sum
        identity = self.downsample is None and self.stride == 1
        link = ShortcutLink() if fused and (identity or self.downsample is not None) else None
        out = self._gemm_bn(xm, self.conv1, self.bn1, relu=True, relu_in=fused and relu_in,
                            link=link, role=1)
        P = out.shape[1]
        self._tap("r1", out.view(R, H, W, P), nhwc=True)
        if fused and P % 256 == 0 and _lib.env("TLOD_HEAD_IMPLICIT", "1") != "0":
            # conv2 as implicit GEMMs over the channels-last map (no im2col / col2im passes);
            # conv1's ReLU backward runs in conv2's input-gradient epilogue (relu_in)
            out = self._gemm_bn(out, self.conv2, self.bn2, relu=True, relu_in=True,
                                nhwc3=(R, H, W))
        else:
            taps = im2col3x3_nhwc(out, (R, H, W), relu_in=fused)
            out = self._gemm_bn(taps, self.conv2, self.bn2, relu=True)
        self._tap("r2", out.view(R, H, W, P), nhwc=True)
        res = (self._gemm_bn(xm, self.downsample[0], self.downsample[1], relu=False,
                             link=link, role=4)
               if self.downsample is not None else xm)
        fuse_mean = mean and fused and self.act_tap is None
        out = self._gemm_bn(out, self.conv3, self.bn3, relu=True, residual=res, relu_in=fused,
                            link=link if identity else None, role=3 if identity else 0,
                            mean_hw=(R, H, W) if fuse_mean else None)
        if fuse_mean:
            return out, None
        self._tap("r3", out.view(R, H, W, -1), nhwc=True)
        return out, (R, H, W)


class ResNetBase(nn.Sequential):
    """RCNN_base = Sequential(conv1, bn1, relu, maxpool, layer1, layer2, layer3).  Slices
    (MAF/ATF taps: [:5] conv1..layer1, [5:6] layer2, [6:] layer3) keep this forward."""

    # split points (shared frozen prefix end, conv3 end, conv4 end) for the MAF / ATF taps
    SPLITS = (5, 5, 6)

    def forward(self, x):
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv2d):  # stem conv1 + bn1 + relu, fused
                assert isinstance(mods[i + 1], nn.BatchNorm2d) and isinstance(mods[i + 2], nn.ReLU)
                x = stem(x, m, mods[i + 1])
                i += 3
                continue
            if isinstance(m, nn.MaxPool2d):
                x = F.max_pool2d(x, m.kernel_size, m.stride, m.padding, ceil_mode=m.ceil_mode)
            else:
                x = m(x)
            i += 1
        return x


class HeadEntry:
    """pool5 as RCNN_top reads it: the channels-last bins (2i, 2j) of RoIAlignAvg (R, QH, QW,
    C) — layer4's first bottleneck subsamples by 2, so the rest of the 7 x 7 map is never
    read (tlod.roi_align.roi_align_avg_s2_nhwc).  Returned by the ResNet models' _pool,
    consumed only by their _head_to_tail."""

    __slots__ = ("x",)

    def __init__(self, x):
        self.x = x


def resnet_pool(model, feat, rois, base_pool):
    """The ResNet detectors' _pool: the head entry for RoIAlignAvg (POOLING_MODE 'align'),
    else the generic pooling (base_pool: the base class's _pool)."""
    ra = model.RCNN_roi_align
    first = model.RCNN_top[0][0]
    if (cfg.POOLING_MODE == "align" and ra.aligned_height <= 7 and ra.aligned_width <= 7
            and first.stride == 2 and _lib.env("TLOD_ROI_HEAD_ENTRY", "1") != "0"):
        from ..roi_align import roi_align_avg_s2_nhwc
        return HeadEntry(roi_align_avg_s2_nhwc(feat, rois, ra.aligned_height, ra.aligned_width,
                                               ra.spatial_scale))
    return base_pool(model, feat, rois)


class ResNetTop(nn.Sequential):
    """RCNN_top = Sequential(layer4); forward(pool5 NCHW, or the HeadEntry) -> channels-last
    features."""

    def forward(self, pool5, mean=False):
        """mean: return fc7 = out.mean(3).mean(2) of the NCHW reference (resnet.py:286-288),
        (R, C), taken in the last GEMM function when it can (LinearActFunction mean_hw)."""
        if isinstance(pool5, HeadEntry):
            x, sub = pool5.x, True
        else:
            x, sub = pool5.permute(0, 2, 3, 1), False
        shape = None
        blocks = list(self[0])
        for i, block in enumerate(blocks):
            x, shape = block.forward_nhwc(x, subsampled=sub and i == 0, shape=shape,
                                          relu_in=shape is not None,
                                          mean=mean and i == len(blocks) - 1)
            if shape is None:  # the mean was taken by the last block
                return x
        y = x.view(*shape, x.shape[-1])
        return head_mean(y) if mean else y


class HeadMeanFunction(torch.autograd.Function):
    """fc7 = RCNN_top(pool5).mean(3).mean(2) (lib/DAF/resnet.py:286-288) on the channels-last
    head output (R, H, W, C): the same two means forward; the backward returns (g / H) / W
    (the order of autograd's two mean backwards) broadcast as a stride-0 view — autograd's chain materialises it twice (one (R, H, C) and
    one (R, H, W, C) division) before the last bottleneck's ReLU mask reads it, which takes
    the view directly (LinearActFunction)."""

    @staticmethod
    def forward(ctx, y):
        ctx.shape = y.shape
        return y.mean(2).mean(1)

    @staticmethod
    def backward(ctx, g):
        R, H, W, C = ctx.shape
        return ((g / H) / W)[:, None, None, :].expand(R, H, W, C)


def head_mean(y):
    return HeadMeanFunction.apply(y)


def _make_layer(inplanes, planes, blocks, stride=1):
    downsample = None
    if stride != 1 or inplanes != planes * 4:
        downsample = nn.Sequential(
            nn.Conv2d(inplanes, planes * 4, kernel_size=1, stride=stride, bias=False),
            nn.BatchNorm2d(planes * 4))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * 4, planes))
    return nn.Sequential(*layers)


def resnet101_parts(fixed_blocks=1):
    """(RCNN_base, RCNN_top) of resnet101() with the reference init (resnet.py:120-128:
    conv N(0, sqrt(2/(k*k*out))), BN weight 1 / bias 0) and freezing (:249-267)."""
    conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
    bn1 = nn.BatchNorm2d(64)
    maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=0, ceil_mode=True)
    layer1 = _make_layer(64, 64, 3)
    layer2 = _make_layer(256, 128, 4, stride=2)
    layer3 = _make_layer(512, 256, 23, stride=2)
    layer4 = _make_layer(1024, 512, 3, stride=2)
    base = ResNetBase(conv1, bn1, nn.ReLU(inplace=True), maxpool, layer1, layer2, layer3)
    top = ResNetTop(layer4)
    for m in list(base.modules()) + list(top.modules()):
        if isinstance(m, nn.Conv2d):
            n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
            m.weight.data.normal_(0, math.sqrt(2.0 / n))
        elif isinstance(m, nn.BatchNorm2d):
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    for p in list(base[0].parameters()) + list(base[1].parameters()):
        p.requires_grad = False
    assert 0 <= fixed_blocks < 4
    for idx in range(4, 4 + fixed_blocks):  # layer1 (.. layer3)
        for p in base[idx].parameters():
            p.requires_grad = False
    for m in list(base.modules()) + list(top.modules()):
        if isinstance(m, nn.BatchNorm2d):
            for p in m.parameters():
                p.requires_grad = False
    return base, top


def set_bn_eval(module):
    """resnet.py:269-284: BatchNorm always in eval mode (frozen running statistics)."""
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.eval()
