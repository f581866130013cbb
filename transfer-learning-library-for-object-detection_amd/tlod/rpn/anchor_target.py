"""Drop-in ``_AnchorTargetLayer`` (lib/model/rpn/anchor_target_layer.py:29-219).

forward((rpn_cls_score, gt_boxes, im_info, num_boxes)) ->
    [labels (B,1,A*H,W), bbox_targets (B,4A,H,W), inside_w (B,4A,H,W), outside_w (B,4A,H,W)]

Production mode (default): both libtlod phases back to back, subsampling drawn by the
device RNG (seeded per call from ``seed`` and a call counter) — no host sync.
Replay mode (``rng=`` an object with ``permutation(n)``, e.g. ``np.random``): the label
phase runs, the host reads the fg/bg counts, draws the permutations exactly where the
reference does (:131, :143) and feeds them to the sampling phase — the bit-exact parity
path used by the tests.
"""
import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from ..config import cfg
from .anchors import base_anchor_tensor


def rpn_cfg_struct(c=None):
    c = c or cfg.TRAIN
    return _lib.RpnCfg(float(c.RPN_POSITIVE_OVERLAP), float(c.RPN_NEGATIVE_OVERLAP),
                       float(c.RPN_FG_FRACTION), int(c.RPN_BATCHSIZE),
                       int(bool(c.RPN_CLOBBER_POSITIVES)), float(c.RPN_BBOX_INSIDE_WEIGHTS[0]), 0)


class _AnchorTargetLayer(nn.Module):
    def __init__(self, feat_stride, scales, ratios, seed=None):
        super().__init__()
        self._feat_stride = int(feat_stride)
        self._scales = scales
        self.register_buffer("_anchors", base_anchor_tensor(scales, ratios), persistent=False)
        self._num_anchors = self._anchors.size(0)
        self._allowed_border = 0
        self.seed = int(cfg.RNG_SEED if seed is None else seed)
        self.calls = 0

    def forward(self, input, rng=None):
        rpn_cls_score, gt_boxes, im_info, _num_boxes = input
        H, W = rpn_cls_score.shape[2], rpn_cls_score.shape[3]
        self.calls += 1
        return anchor_target(self._anchors, H, W, self._feat_stride, gt_boxes, im_info,
                             rpn_cfg_struct(), rng=rng,
                             seed=(self.seed * 1000003 + self.calls) & 0xFFFFFFFFFFFFFFFF)


def anchor_target(base_anchors, H, W, feat_stride, gt_boxes, im_info, cfg_struct, rng=None,
                  seed=0):
    _lib.require_cuda(gt_boxes, im_info)
    dev = gt_boxes.device
    gt = gt_boxes.detach().contiguous().float()
    info = im_info.detach().contiguous().float()
    anchors = base_anchors.to(dev).contiguous()
    B, G = gt.shape[0], gt.shape[1]
    A = anchors.shape[0]
    L = _lib.lib()
    ws = _lib.workspace(L.tlod_anchor_target_workspace_bytes(B, A, H, W, G), dev, "anchor_target")
    counts = torch.empty(2 * B, dtype=torch.int32, device=dev)
    labels = torch.empty((B, 1, A * H, W), dtype=torch.float32, device=dev)
    targets = torch.empty((B, 4 * A, H, W), dtype=torch.float32, device=dev)
    inside = torch.empty_like(targets)
    outside = torch.empty_like(targets)
    s = _lib.stream_of(gt)
    cs = cfg_struct
    if rng is None:
        _lib.check(L.tlod_anchor_target_f32(
            _lib.ptr(anchors), A, H, W, feat_stride, _lib.ptr(gt), B, G, _lib.ptr(info),
            cs, seed, _lib.ptr(counts), _lib.ptr(labels), _lib.ptr(targets), _lib.ptr(inside),
            _lib.ptr(outside), _lib.ptr(ws), ws.numel(), s), "anchor_target")
        return [labels, targets, inside, outside]
    # replay mode: reproduce the reference's numpy draws (anchor_target_layer.py:123-145)
    _lib.check(L.tlod_anchor_target_label_f32(
        _lib.ptr(anchors), A, H, W, feat_stride, _lib.ptr(gt), B, G, _lib.ptr(info), cs,
        _lib.ptr(counts), _lib.ptr(ws), ws.numel(), s), "anchor_target_label")
    cnt = counts.cpu().numpy().reshape(B, 2)
    num_fg = int(cs.fg_fraction * cs.batch_size)
    draws, offs = [], [0]
    for b in range(B):
        nfg, nbg = int(cnt[b, 0]), int(cnt[b, 1])
        if nfg > num_fg:
            draws.append(np.asarray(rng.permutation(nfg), dtype=np.int32))
        offs.append(offs[-1] + (len(draws[-1]) if nfg > num_fg else 0))
        num_bg = cs.batch_size - min(nfg, num_fg)
        if nbg > num_bg:
            draws.append(np.asarray(rng.permutation(nbg), dtype=np.int32))
        offs.append(offs[-1] + (len(draws[-1]) if nbg > num_bg else 0))
    flat = np.concatenate(draws) if draws else np.zeros(1, np.int32)
    perm = torch.from_numpy(flat).to(dev)
    perm_off = torch.tensor(offs, dtype=torch.int32, device=dev)
    _lib.check(L.tlod_anchor_target_sample_f32(
        _lib.ptr(anchors), A, H, W, feat_stride, _lib.ptr(gt), B, G, cs, _lib.ptr(perm),
        _lib.ptr(perm_off), 0, _lib.ptr(labels), _lib.ptr(targets), _lib.ptr(inside),
        _lib.ptr(outside), _lib.ptr(ws), ws.numel(), s), "anchor_target_sample")
    torch.cuda.current_stream(dev).synchronize()  # keep perm alive until consumed
    return [labels, targets, inside, outside]
