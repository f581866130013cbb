"""Drop-in ``_ProposalLayer`` (lib/model/rpn/proposal_layer.py:24-175).

forward((rpn_cls_prob, rpn_bbox_pred, im_info, cfg_key)) -> rois (B, post_nms, 5).
One libtlod call (``tlod_proposal_f32``) does decode, clip, sort, pre-NMS top-N, NMS
and post-NMS top-N for every image on the device; no host synchronisation.
"""
import torch
import torch.nn as nn

from .. import _lib
from ..config import cfg
from .anchors import base_anchor_tensor


class _ProposalLayer(nn.Module):
    def __init__(self, feat_stride, scales, ratios):
        super().__init__()
        self._feat_stride = int(feat_stride)
        self.register_buffer("_anchors", base_anchor_tensor(scales, ratios), persistent=False)
        self._num_anchors = self._anchors.size(0)

    def forward(self, input):
        prob, deltas, im_info, cfg_key = input
        c = cfg[cfg_key]
        return proposal(prob, deltas, im_info, self._anchors, self._feat_stride,
                        c.RPN_PRE_NMS_TOP_N, c.RPN_POST_NMS_TOP_N, c.RPN_NMS_THRESH)

    def backward(self, top, propagate_down, bottom):  # proposal_layer.py:163-165
        pass

    def reshape(self, bottom, top):
        pass


def proposal(prob, deltas, im_info, base_anchors, feat_stride, pre_nms, post_nms, nms_thresh,
             return_props=False):
    _lib.require_cuda(prob, deltas, im_info)
    prob = prob.detach().contiguous().float()
    deltas = deltas.detach().contiguous().float()
    im_info = im_info.detach().contiguous().float()
    anchors = base_anchors.to(prob.device).contiguous()
    B, twoA, H, W = prob.shape
    A = twoA // 2
    assert deltas.shape == (B, 4 * A, H, W), (deltas.shape, prob.shape)
    L = _lib.lib()
    rois = torch.empty((B, int(post_nms), 5), dtype=torch.float32, device=prob.device)
    props = (torch.empty((B, H * W * A, 4), dtype=torch.float32, device=prob.device)
             if return_props else None)
    ws = _lib.workspace(L.tlod_proposal_workspace_bytes(B, A, H, W, int(pre_nms)), prob.device,
                        "proposal")
    _lib.check(L.tlod_proposal_f32(
        _lib.ptr(prob), _lib.ptr(deltas), _lib.ptr(im_info), _lib.ptr(anchors), B, A, H, W,
        int(feat_stride), int(pre_nms), int(post_nms), float(nms_thresh), _lib.ptr(rois),
        _lib.ptr(props), _lib.ptr(ws), ws.numel(), _lib.stream_of(prob)), "proposal")
    return (rois, props) if return_props else rois
