"""Drop-in for ``model.roi_pooling`` (lib/model/roi_pooling/{functions,modules}/roi_pool.py).

``_RoIPooling(pooled_height, pooled_width, spatial_scale)`` as in modules/roi_pool.py:5-14.
Forward keeps the int32 argmax (flat input index, -1 if empty) like the reference; the
backward scatters through it in libtlod instead of the reference's per-input gather.
"""
import torch
from torch.nn import Module

from . import _lib


class RoIPoolFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, rois, pooled_height, pooled_width, spatial_scale):
        _lib.require_cuda(features, rois)
        feat = features.contiguous()
        rois_c = rois.contiguous().float()
        B, C, H, W = feat.shape
        R = rois_c.shape[0]
        ph, pw = int(pooled_height), int(pooled_width)
        out = torch.empty((R, C, ph, pw), dtype=feat.dtype, device=feat.device)
        argmax = torch.empty((R, C, ph, pw), dtype=torch.int32, device=feat.device)
        _lib.check(_lib.lib().tlod_roi_pool_fwd_f32(
            _lib.ptr(feat), B, C, H, W, _lib.ptr(rois_c), R, ph, pw, float(spatial_scale),
            _lib.ptr(out), _lib.ptr(argmax), _lib.stream_of(feat)), "roi_pool_fwd")
        ctx.save_for_backward(argmax)
        ctx.meta = (B, C, H, W)
        ctx.mark_non_differentiable(argmax)
        return out, argmax

    @staticmethod
    def backward(ctx, grad_output, _grad_argmax=None):
        (argmax,) = ctx.saved_tensors
        B, C, H, W = ctx.meta
        g = grad_output.contiguous()
        R, _, ph, pw = g.shape
        grad_in = torch.zeros((B, C, H, W), dtype=g.dtype, device=g.device)
        _lib.check(_lib.lib().tlod_roi_pool_bwd_f32(
            _lib.ptr(g), _lib.ptr(argmax), R, C, ph, pw, _lib.ptr(grad_in), _lib.stream_of(g)),
            "roi_pool_bwd")
        return grad_in, None, None, None, None


class _RoIPooling(Module):
    def __init__(self, pooled_height, pooled_width, spatial_scale):
        super().__init__()
        self.pooled_width = int(pooled_width)
        self.pooled_height = int(pooled_height)
        self.spatial_scale = float(spatial_scale)

    def forward(self, features, rois):
        out, _ = RoIPoolFunction.apply(features, rois, self.pooled_height, self.pooled_width,
                                       self.spatial_scale)
        return out


def roi_pool_with_argmax(features, rois, pooled_height, pooled_width, spatial_scale):
    """(out, argmax) — exposes the argmax for parity tests."""
    return RoIPoolFunction.apply(features, rois, pooled_height, pooled_width, spatial_scale)
