"""Drop-ins for ``model.roi_align`` (lib/model/roi_align/{functions,modules}/roi_align.py).

``RoIAlign``, ``RoIAlignAvg`` and ``RoIAlignMax`` keep the reference constructors
``(aligned_height, aligned_width, spatial_scale)``.  Forward/backward run in libtlod
(``tlod_roi_align_*_f32``); RoIAlignAvg uses the fused align+avg-pool kernels.
The reference's CPU path (roi_align.c, with an inverted bounds test at :175) is not
reproduced: inputs must be CUDA tensors.
"""
import torch
import torch.nn.functional as F
from torch.nn import Module

from . import _lib


class RoIAlignFunction(torch.autograd.Function):
    """functions/roi_align.py:7-51 as a static autograd Function."""

    @staticmethod
    def forward(ctx, features, rois, aligned_height, aligned_width, spatial_scale):
        _lib.require_cuda(features, rois)
        feat = features.contiguous()
        rois_c = rois.contiguous().float()
        B, C, H, W = feat.shape
        R = rois_c.shape[0]
        ah, aw, sc = int(aligned_height), int(aligned_width), float(spatial_scale)
        out = torch.empty((R, C, ah, aw), dtype=feat.dtype, device=feat.device)
        _lib.check(_lib.lib().tlod_roi_align_fwd_f32(
            _lib.ptr(feat), B, C, H, W, _lib.ptr(rois_c), R, ah, aw, sc, _lib.ptr(out),
            _lib.stream_of(feat)), "roi_align_fwd")
        ctx.save_for_backward(rois_c)
        ctx.meta = (B, C, H, W, ah, aw, sc)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (rois_c,) = ctx.saved_tensors
        B, C, H, W, ah, aw, sc = ctx.meta
        g = grad_output.contiguous()
        grad_in = torch.zeros((B, C, H, W), dtype=g.dtype, device=g.device)
        _lib.check(_lib.lib().tlod_roi_align_bwd_f32(
            _lib.ptr(g), B, C, H, W, _lib.ptr(rois_c), rois_c.shape[0], ah, aw, sc,
            _lib.ptr(grad_in), _lib.stream_of(g)), "roi_align_bwd")
        return grad_in, None, None, None, None


class RoIAlignAvgFunction(torch.autograd.Function):
    """RoIAlignAvg fused: align at (ph+1, pw+1) + avg_pool2d(2, 1) (modules/roi_align.py:18-29)."""

    @staticmethod
    def forward(ctx, features, rois, pooled_height, pooled_width, spatial_scale):
        _lib.require_cuda(features, rois)
        feat = features.contiguous()
        rois_c = rois.contiguous().float()
        B, C, H, W = feat.shape
        R = rois_c.shape[0]
        ph, pw, sc = int(pooled_height), int(pooled_width), float(spatial_scale)
        out = torch.empty((R, C, ph, pw), dtype=feat.dtype, device=feat.device)
        _lib.check(_lib.lib().tlod_roi_align_avg_fwd_f32(
            _lib.ptr(feat), B, C, H, W, _lib.ptr(rois_c), R, ph, pw, sc, _lib.ptr(out),
            _lib.stream_of(feat)), "roi_align_avg_fwd")
        ctx.save_for_backward(rois_c)
        ctx.meta = (B, C, H, W, ph, pw, sc)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (rois_c,) = ctx.saved_tensors
        B, C, H, W, ph, pw, sc = ctx.meta
        g = grad_output.contiguous()
        grad_in = torch.zeros((B, C, H, W), dtype=g.dtype, device=g.device)
        L = _lib.lib()
        R = rois_c.shape[0]
        ws = _lib.workspace(max(L.tlod_roi_align_avg_bwd_gather_workspace_bytes(B, C, H, W, R, ph, pw),
                                L.tlod_roi_align_avg_bwd_workspace_bytes(B, C, H, W)), g.device,
                            "roi_align_bwd")
        _lib.check(L.tlod_roi_align_avg_bwd_f32(
            _lib.ptr(g), B, C, H, W, _lib.ptr(rois_c), rois_c.shape[0], ph, pw, sc,
            _lib.ptr(grad_in), _lib.ptr(ws), ws.numel(), _lib.stream_of(g)), "roi_align_avg_bwd")
        return grad_in, None, None, None, None


class RoIAlignAvgS2Function(torch.autograd.Function):
    """The ResNet RoI head's entry: RoIAlignAvg bins (2i, 2j), channels-last (R, QH, QW, C)
    (tlod_roi_align_avg_s2_nhwc_*_f32) — RCNN_top = layer4 subsamples pool5 by 2 in its first
    bottleneck (lib/DAF/resnet.py:64-102), so the other bins, the 7 x 7 map and its
    channels-last permute are never needed.  Equal bit for bit to
    RoIAlignAvgFunction(...).permute(0, 2, 3, 1)[:, ::2, ::2, :] and its gradient."""

    @staticmethod
    def forward(ctx, features, rois, pooled_height, pooled_width, spatial_scale):
        _lib.require_cuda(features, rois)
        feat = features.contiguous()
        rois_c = rois.contiguous().float()
        B, C, H, W = feat.shape
        R = rois_c.shape[0]
        ph, pw, sc = int(pooled_height), int(pooled_width), float(spatial_scale)
        out = torch.empty((R, (ph + 1) // 2, (pw + 1) // 2, C), dtype=feat.dtype,
                          device=feat.device)
        L = _lib.lib()
        ws = _lib.workspace(L.tlod_roi_align_avg_s2_workspace_bytes(B, C, H, W, max(R, 1), ph, pw),
                            feat.device, "roi_align_s2")
        _lib.check(L.tlod_roi_align_avg_s2_nhwc_fwd_f32(
            _lib.ptr(feat), B, C, H, W, _lib.ptr(rois_c), R, ph, pw, sc, _lib.ptr(out),
            _lib.ptr(ws), ws.numel(), _lib.stream_of(feat)), "roi_align_avg_s2_nhwc_fwd")
        ctx.save_for_backward(rois_c)
        ctx.meta = (B, C, H, W, ph, pw, sc)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (rois_c,) = ctx.saved_tensors
        B, C, H, W, ph, pw, sc = ctx.meta
        g = grad_output.contiguous()
        R = rois_c.shape[0]
        grad_in = torch.zeros((B, C, H, W), dtype=g.dtype, device=g.device)
        L = _lib.lib()
        ws = _lib.workspace(L.tlod_roi_align_avg_s2_workspace_bytes(B, C, H, W, max(R, 1), ph, pw),
                            g.device, "roi_align_s2")
        _lib.check(L.tlod_roi_align_avg_s2_nhwc_bwd_f32(
            _lib.ptr(g), B, C, H, W, _lib.ptr(rois_c), R, ph, pw, sc, _lib.ptr(grad_in),
            _lib.ptr(ws), ws.numel(), _lib.stream_of(g)), "roi_align_avg_s2_nhwc_bwd")
        return grad_in, None, None, None, None


def roi_align_avg_s2_nhwc(features, rois, pooled_height, pooled_width, spatial_scale):
    return RoIAlignAvgS2Function.apply(features, rois, pooled_height, pooled_width, spatial_scale)


class RoIAlign(Module):
    def __init__(self, aligned_height, aligned_width, spatial_scale):
        super().__init__()
        self.aligned_width = int(aligned_width)
        self.aligned_height = int(aligned_height)
        self.spatial_scale = float(spatial_scale)

    def forward(self, features, rois):
        return RoIAlignFunction.apply(features, rois, self.aligned_height, self.aligned_width,
                                      self.spatial_scale)


class RoIAlignAvg(RoIAlign):
    def forward(self, features, rois):
        if self.aligned_height <= 7 and self.aligned_width <= 7:
            return RoIAlignAvgFunction.apply(features, rois, self.aligned_height,
                                             self.aligned_width, self.spatial_scale)
        x = RoIAlignFunction.apply(features, rois, self.aligned_height + 1,
                                   self.aligned_width + 1, self.spatial_scale)
        return F.avg_pool2d(x, kernel_size=2, stride=1)


class RoIAlignMax(RoIAlign):
    def forward(self, features, rois):
        x = RoIAlignFunction.apply(features, rois, self.aligned_height + 1,
                                   self.aligned_width + 1, self.spatial_scale)
        return F.max_pool2d(x, kernel_size=2, stride=1)
