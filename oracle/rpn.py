"""Oracle: RPN proposal layer, anchor-target and proposal-target layers (test infra only).

Randomness: the reference draws ``np.random.permutation`` / ``np.random.rand`` from the
global numpy RNG (anchor_target_layer.py:131,143; proposal_target_layer_cascade.py:158,
167,174,182).  Here every draw goes through an ``rng`` object with ``permutation(n)`` and
``rand(n)`` (``np.random`` itself, or a RandomState, or a recorder) so tests can replay
the identical draws into the HIP path's explicit-permutation inputs.
"""
import numpy as np

from .boxes import (bbox_overlaps, bbox_transform, bbox_transform_inv, clip_boxes,
                    generate_anchors, shifted_anchors)
from .nms import nms

f32 = np.float32


class Recorder:
    """Wraps a numpy RandomState and records every draw in call order."""

    def __init__(self, seed_or_state):
        self.rs = (seed_or_state if isinstance(seed_or_state, np.random.RandomState)
                   else np.random.RandomState(seed_or_state))
        self.log = []

    def permutation(self, n):
        p = self.rs.permutation(n)
        self.log.append(("perm", p.copy()))
        return p

    def rand(self, n):
        u = self.rs.rand(n)
        self.log.append(("rand", u.copy()))
        return u


# ------------------------------------------------------------- proposal layer
def proposal_layer(cls_prob, bbox_deltas, im_info, base_anchors, feat_stride,
                   pre_nms, post_nms, nms_thresh):
    """_ProposalLayer.forward (lib/model/rpn/proposal_layer.py:49-161).

    cls_prob (B,2A,H,W) [bg A | fg A], bbox_deltas (B,4A,H,W), im_info (B,3).
    Sort: stable descending (torch.sort at :125 is unstable; ties are measure-zero on
    real scores, the build pins the stable order).  No min-size filter (:113 disabled).
    Returns rois (B, post_nms, 5) float32, zero-padded, column 0 = batch index.
    """
    B, twoA, H, W = cls_prob.shape
    A = base_anchors.shape[0]
    scores = cls_prob[:, A:].transpose(0, 2, 3, 1).reshape(B, -1).astype(np.float32)
    deltas = bbox_deltas.transpose(0, 2, 3, 1).reshape(B, -1, 4).astype(np.float32)
    anchors = shifted_anchors(base_anchors, H, W, feat_stride)
    out = np.zeros((B, post_nms, 5), np.float32)
    for i in range(B):
        props = clip_boxes(bbox_transform_inv(anchors, deltas[i]), im_info[i, 0], im_info[i, 1])
        order = np.argsort(-scores[i], kind="stable")
        if 0 < pre_nms < scores.size:                 # numel over the whole batch (:135)
            order = order[:pre_nms]
        p = props[order]
        s = scores[i][order]
        keep = nms(np.concatenate([p, s[:, None]], 1), nms_thresh,
                   max_keep=post_nms if post_nms > 0 else None)
        if post_nms > 0:
            keep = keep[:post_nms]
        out[i, :, 0] = i
        out[i, :len(keep), 1:] = p[keep]
    return out


def decode_clip(cls_prob, bbox_deltas, im_info, base_anchors, feat_stride):
    """The decode+clip half of proposal_layer (:78-109): returns (scores (B,N), props (B,N,4))."""
    B, twoA, H, W = cls_prob.shape
    A = base_anchors.shape[0]
    scores = cls_prob[:, A:].transpose(0, 2, 3, 1).reshape(B, -1).astype(np.float32)
    deltas = bbox_deltas.transpose(0, 2, 3, 1).reshape(B, -1, 4).astype(np.float32)
    anchors = shifted_anchors(base_anchors, H, W, feat_stride)
    props = np.stack([clip_boxes(bbox_transform_inv(anchors, deltas[i]), im_info[i, 0], im_info[i, 1])
                      for i in range(B)])
    return scores, props


# ------------------------------------------------------------- anchor target
DEFAULT_RPN = dict(pos=0.7, neg=0.3, fg_frac=0.5, batch=256, clobber=False,
                   inside_w=1.0, pos_weight=-1.0, border=0)


def anchor_target(feat_h, feat_w, gt_boxes, im_info, base_anchors, feat_stride, rng,
                  cfg=DEFAULT_RPN):
    """_AnchorTargetLayer.forward (lib/model/rpn/anchor_target_layer.py:48-193).

    gt_boxes (B,G,5) float32, im_info (B,3).  Returns [labels (B,1,A*H,W),
    bbox_targets (B,4A,H,W), inside_w (B,4A,H,W), outside_w (B,4A,H,W)] float32.
    """
    B = gt_boxes.shape[0]
    A = base_anchors.shape[0]
    K = feat_h * feat_w
    total = K * A
    all_anchors = shifted_anchors(base_anchors, feat_h, feat_w, feat_stride)
    brd = cfg["border"]
    keep = ((all_anchors[:, 0] >= -brd) & (all_anchors[:, 1] >= -brd) &
            (all_anchors[:, 2] < int(im_info[0][1]) + brd) &
            (all_anchors[:, 3] < int(im_info[0][0]) + brd))          # :83-87 (image 0's size)
    inds_inside = np.nonzero(keep)[0]
    anchors = all_anchors[inds_inside]
    n = len(inds_inside)
    labels = np.full((B, n), -1, np.float32)
    biw = np.zeros((B, n), np.float32)
    bow = np.zeros((B, n), np.float32)
    overlaps = np.stack([bbox_overlaps(anchors, gt_boxes[b]) for b in range(B)])   # (B,n,G)
    max_ov = overlaps.max(2)
    argmax_ov = overlaps.argmax(2)
    gt_max = overlaps.max(1)                                                      # (B,G)
    if not cfg["clobber"]:
        labels[max_ov < f32(cfg["neg"])] = 0
    gt_max[gt_max == 0] = f32(1e-5)
    keepc = (overlaps == gt_max[:, None, :]).sum(2)
    labels[keepc > 0] = 1
    labels[max_ov >= f32(cfg["pos"])] = 1
    if cfg["clobber"]:
        labels[max_ov < f32(cfg["neg"])] = 0
    num_fg = int(cfg["fg_frac"] * cfg["batch"])
    sum_fg = (labels == 1).sum(1)
    sum_bg = (labels == 0).sum(1)
    for i in range(B):                                                            # :123-145
        if sum_fg[i] > num_fg:
            fg_inds = np.nonzero(labels[i] == 1)[0]
            p = rng.permutation(len(fg_inds))
            labels[i][fg_inds[p[:len(fg_inds) - num_fg]]] = -1
        num_bg = cfg["batch"] - int((labels == 1).sum(1)[i])
        if sum_bg[i] > num_bg:
            bg_inds = np.nonzero(labels[i] == 0)[0]
            p = rng.permutation(len(bg_inds))
            labels[i][bg_inds[p[:len(bg_inds) - num_bg]]] = -1
    targets = np.stack([bbox_transform(anchors, gt_boxes[b][argmax_ov[b], :4]) for b in range(B)])
    biw[labels == 1] = f32(cfg["inside_w"])
    assert cfg["pos_weight"] < 0
    num_examples = int((labels[B - 1] >= 0).sum())   # uses the loop's last i (:154)
    w = f32(1.0 / num_examples)
    bow[labels == 1] = w
    bow[labels == 0] = w

    def unmap(d, fill):
        ret = np.full((B, total) + d.shape[2:], fill, np.float32)
        ret[:, inds_inside] = d
        return ret

    labels = unmap(labels, -1)
    targets = unmap(targets, 0)
    biw = unmap(biw, 0)
    bow = unmap(bow, 0)
    H, W = feat_h, feat_w
    labels = labels.reshape(B, H, W, A).transpose(0, 3, 1, 2).reshape(B, 1, A * H, W)
    targets = targets.reshape(B, H, W, 4 * A).transpose(0, 3, 1, 2)
    biw = np.repeat(biw[:, :, None], 4, 2).reshape(B, H, W, 4 * A).transpose(0, 3, 1, 2)
    bow = np.repeat(bow[:, :, None], 4, 2).reshape(B, H, W, 4 * A).transpose(0, 3, 1, 2)
    return [np.ascontiguousarray(x, dtype=np.float32) for x in (labels, targets, biw, bow)]


# ------------------------------------------------------------- proposal target
DEFAULT_RCNN = dict(batch=256, fg_frac=0.25, fg_thresh=0.5, bg_hi=0.5, bg_lo=0.0,
                    means=(0.0, 0.0, 0.0, 0.0), stds=(0.1, 0.1, 0.2, 0.2),
                    inside_w=(1.0, 1.0, 1.0, 1.0))


def proposal_target(rois, gt_boxes, rng, cfg=DEFAULT_RCNN):
    """_ProposalTargetLayer.forward (lib/model/rpn/proposal_target_layer_cascade.py:33-212).

    rois (B,R,5), gt_boxes (B,G,5).  Returns (rois (B,S,5), labels (B,S), targets (B,S,4),
    inside_w (B,S,4), outside_w (B,S,4)), S = cfg batch (256 with cfgs/vgg16.yml).
    """
    B, R, _ = rois.shape
    G = gt_boxes.shape[1]
    gt_append = np.zeros_like(gt_boxes, dtype=np.float32)
    gt_append[:, :, 1:5] = gt_boxes[:, :, :4]
    all_rois = np.concatenate([rois.astype(np.float32), gt_append], 1)          # :39-43
    S = int(cfg["batch"])
    fg_per = int(np.round(cfg["fg_frac"] * S))
    fg_per = 1 if fg_per == 0 else fg_per
    labels_b = np.zeros((B, S), np.float32)
    rois_b = np.zeros((B, S, 5), np.float32)
    gt_rois_b = np.zeros((B, S, 5), np.float32)
    for i in range(B):
        ov = bbox_overlaps(all_rois[i, :, 1:5], gt_boxes[i])                    # :122
        max_ov = ov.max(1)
        assign = ov.argmax(1)
        labels = gt_boxes[i, assign, 4]
        fg_inds = np.nonzero(max_ov >= f32(cfg["fg_thresh"]))[0]
        bg_inds = np.nonzero((max_ov < f32(cfg["bg_hi"])) & (max_ov >= f32(cfg["bg_lo"])))[0]
        nfg, nbg = len(fg_inds), len(bg_inds)
        if nfg > 0 and nbg > 0:
            fg_this = min(fg_per, nfg)
            p = rng.permutation(nfg)
            fg_inds = fg_inds[p[:fg_this]]
            bg_this = S - fg_this
            rn = np.floor(rng.rand(bg_this) * nbg).astype(np.int64)
            bg_inds = bg_inds[rn]
        elif nfg > 0 and nbg == 0:
            rn = np.floor(rng.rand(S) * nfg).astype(np.int64)
            fg_inds = fg_inds[rn]
            fg_this = S
        elif nbg > 0 and nfg == 0:
            rn = np.floor(rng.rand(S) * nbg).astype(np.int64)
            bg_inds = bg_inds[rn]
            fg_this = 0
            fg_inds = fg_inds[:0]
        else:
            raise ValueError("bg_num_rois = 0 and fg_num_rois = 0, this should not happen!")
        keep = np.concatenate([fg_inds, bg_inds]) if fg_this < S else fg_inds
        labels_b[i] = labels[keep]
        if fg_this < S:
            labels_b[i][fg_this:] = 0
        rois_b[i] = all_rois[i][keep]
        rois_b[i, :, 0] = i
        gt_rois_b[i] = gt_boxes[i][assign[keep]]
    t = np.stack([bbox_transform(rois_b[i, :, 1:5], gt_rois_b[i, :, :4]) for i in range(B)])
    means = np.asarray(cfg["means"], np.float32)
    stds = np.asarray(cfg["stds"], np.float32)
    t = ((t - means) / stds).astype(np.float32)                                  # :108-111
    targets = np.zeros((B, S, 4), np.float32)
    biw = np.zeros((B, S, 4), np.float32)
    pos = labels_b > 0
    targets[pos] = t[pos]
    biw[pos] = np.asarray(cfg["inside_w"], np.float32)
    bow = (biw > 0).astype(np.float32)
    return rois_b, labels_b, targets, biw, bow


def make_base_anchors(scales=(4, 8, 16, 32), ratios=(0.5, 1, 2)):
    return generate_anchors(scales=np.array(scales), ratios=np.array(ratios))
