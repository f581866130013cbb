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


_SIDE_STREAMS = {}


def side_stream(device, idx):
    """A cached side stream per (device, slot)."""
    key = (str(device), idx)
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _SIDE_STREAMS[key] = st
    return st


class PendingProposals:
    """Proposal layers running on side streams; ``join()`` makes the caller's stream wait
    for them and returns their rois in submission order."""

    def __init__(self, main, streams, outs):
        self.main, self.streams, self.outs = main, streams, outs

    def join(self):
        for st in self.streams:
            self.main.wait_stream(st)
        for o in self.outs:
            o.record_stream(self.main)
        return self.outs


def proposals_on_side_streams(layer, jobs):
    """Run ``layer((prob, deltas, im_info, cfg_key))`` for each job on its own side stream.

    Scheduling only (same kernels, same results): each proposal layer ends in a greedy NMS
    scan that occupies a single workgroup for 0.03-0.35 ms; on side streams the source
    (TRAIN, 12000 -> 2000) and target (TEST, 6000 -> 300) scans run concurrently with each
    other and with the anchor-target / RPN-loss / image-DA work the caller issues before
    ``join()``."""
    main = torch.cuda.current_stream()
    streams, outs = [], []
    for i, (prob, deltas, info, key) in enumerate(jobs):
        st = side_stream(prob.device, i)
        st.wait_stream(main)
        with torch.cuda.stream(st):
            outs.append(layer((prob, deltas, info, key)))
        for t in (prob, deltas, info):
            t.record_stream(st)
        streams.append(st)
    return PendingProposals(main, streams, outs)


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
