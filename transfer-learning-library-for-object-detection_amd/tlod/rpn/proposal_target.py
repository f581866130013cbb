"""Drop-in ``_ProposalTargetLayer`` (lib/model/rpn/proposal_target_layer_cascade.py:20-212).

forward(all_rois, gt_boxes, num_boxes) -> rois, labels, bbox_targets, inside_w, outside_w
with the reference shapes (B,S,5), (B,S), (B,S,4) x3.  Production mode samples with the
device RNG; replay mode (``rng=``) reads the candidate counts and replays the reference's
``np.random.permutation`` / ``np.random.rand`` draws (:158, :167, :174, :182) exactly.
"""
import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from ..config import cfg


def rcnn_cfg_struct(c=None):
    c = c or cfg.TRAIN
    f4 = _lib.c_float * 4
    return _lib.RcnnCfg(int(c.BATCH_SIZE), float(c.FG_FRACTION), float(c.FG_THRESH),
                        float(c.BG_THRESH_HI), float(c.BG_THRESH_LO),
                        f4(*map(float, c.BBOX_NORMALIZE_MEANS)), f4(*map(float, c.BBOX_NORMALIZE_STDS)),
                        f4(*map(float, c.BBOX_INSIDE_WEIGHTS)))


class _ProposalTargetLayer(nn.Module):
    def __init__(self, nclasses, seed=None):
        super().__init__()
        self._num_classes = nclasses
        self.seed = int(cfg.RNG_SEED if seed is None else seed) + 7919
        self.calls = 0

    def forward(self, all_rois, gt_boxes, num_boxes, rng=None):
        self.calls += 1
        return proposal_target(all_rois, gt_boxes, rcnn_cfg_struct(), rng=rng,
                               seed=(self.seed * 1000003 + self.calls) & 0xFFFFFFFFFFFFFFFF)

    def backward(self, top, propagate_down, bottom):
        pass

    def reshape(self, bottom, top):
        pass


def proposal_target(rois, gt_boxes, cs, rng=None, seed=0):
    _lib.require_cuda(rois, gt_boxes)
    dev = rois.device
    r = rois.detach().contiguous().float()
    gt = gt_boxes.detach().contiguous().float()
    B, R = r.shape[0], r.shape[1]
    G = gt.shape[1]
    S = int(cs.batch_size)
    L = _lib.lib()
    ws = _lib.workspace(L.tlod_proposal_target_workspace_bytes(B, R, G), dev, "proposal_target")
    counts = torch.empty(2 * B, dtype=torch.int32, device=dev)
    rois_out = torch.empty((B, S, 5), dtype=torch.float32, device=dev)
    labels = torch.empty((B, S), dtype=torch.float32, device=dev)
    targets = torch.empty((B, S, 4), dtype=torch.float32, device=dev)
    inside = torch.empty_like(targets)
    outside = torch.empty_like(targets)
    s = _lib.stream_of(r)
    if rng is None:
        _lib.check(L.tlod_proposal_target_f32(
            _lib.ptr(r), B, R, _lib.ptr(gt), G, cs, seed, _lib.ptr(counts), _lib.ptr(rois_out),
            _lib.ptr(labels), _lib.ptr(targets), _lib.ptr(inside), _lib.ptr(outside),
            _lib.ptr(ws), ws.numel(), s), "proposal_target")
        return rois_out, labels, targets, inside, outside
    _lib.check(L.tlod_proposal_target_count_f32(
        _lib.ptr(r), B, R, _lib.ptr(gt), G, cs, _lib.ptr(counts), _lib.ptr(ws), ws.numel(), s),
        "proposal_target_count")
    cnt = counts.cpu().numpy().reshape(B, 2)
    fg_per = int(np.round(cs.fg_fraction * S)) or 1
    perms, poff, rands, roff = [], [0], [], [0]
    for b in range(B):
        nfg, nbg = int(cnt[b, 0]), int(cnt[b, 1])
        if nfg > 0 and nbg > 0:
            fg_this = min(fg_per, nfg)
            perms.append(np.asarray(rng.permutation(nfg), np.int32))
            rands.append(np.asarray(rng.rand(S - fg_this), np.float64))
        elif nfg > 0 or nbg > 0:
            perms.append(np.zeros(0, np.int32))
            rands.append(np.asarray(rng.rand(S), np.float64))
        else:
            raise ValueError("bg_num_rois = 0 and fg_num_rois = 0, this should not happen!")
        poff.append(poff[-1] + len(perms[-1]))
        roff.append(roff[-1] + len(rands[-1]))
    perm = torch.from_numpy(np.concatenate(perms + [np.zeros(1, np.int32)])).to(dev)
    rnd = torch.from_numpy(np.concatenate(rands + [np.zeros(1)])).to(dev)
    poff_t = torch.tensor(poff, dtype=torch.int32, device=dev)
    roff_t = torch.tensor(roff, dtype=torch.int32, device=dev)
    _lib.check(L.tlod_proposal_target_sample_f32(
        _lib.ptr(r), B, R, _lib.ptr(gt), G, cs, _lib.ptr(perm), _lib.ptr(poff_t), _lib.ptr(rnd),
        _lib.ptr(roff_t), 0, _lib.ptr(rois_out), _lib.ptr(labels), _lib.ptr(targets),
        _lib.ptr(inside), _lib.ptr(outside), _lib.ptr(ws), ws.numel(), s), "proposal_target_sample")
    torch.cuda.current_stream(dev).synchronize()
    return rois_out, labels, targets, inside, outside
