"""Oracle: test-time detections of one image (TEST INFRASTRUCTURE ONLY).

Restates methods/DAF/DAF_test.py:279-333 (the same loop is in every method's *_test.py):
deltas * BBOX_NORMALIZE_STDS + MEANS, bbox_transform_inv + clip_boxes (oracle.boxes, the
float32 restatement of lib/model/rpn/bbox_transform.py:77-103 / :125-133), / im_scale,
then per class j >= 1: scores > thresh, descending sort (stable here; the reference's
torch.sort is not, which only matters for exactly tied scores), nms (oracle.nms, the CUDA
kernel's semantics) and the max_per_image cut over all classes.
"""
import numpy as np

from . import boxes as obox
from .nms import nms

STDS = (0.1, 0.1, 0.2, 0.2)
MEANS = (0.0, 0.0, 0.0, 0.0)


def decode(rois, bbox_pred, im_info, n_classes, agnostic=False):
    """(R, C, 4) float32 boxes of every class, in original-image coordinates."""
    f32 = np.float32
    R = rois.shape[0]
    d = bbox_pred.reshape(R, -1, 4).astype(f32)
    d = (d * np.asarray(STDS, f32) + np.asarray(MEANS, f32)).astype(f32)
    out = np.zeros((R, n_classes, 4), f32)
    for j in range(n_classes):
        dj = d[:, 0 if agnostic else j]
        b = obox.bbox_transform_inv(rois[:, 1:5], dj)
        b = obox.clip_boxes(b, im_info[0], im_info[1])
        out[:, j] = (b / f32(im_info[2])).astype(f32)
    return out


def postprocess(boxes, cls_prob, thresh=0.0, nms_thresh=0.3, max_per_image=100):
    """boxes (R, C, 4) as from decode(), cls_prob (R, C) -> list over classes of (n, 5)."""
    R, C = cls_prob.shape
    per_class = [np.zeros((0, 5), np.float32)]
    for j in range(1, C):
        inds = np.nonzero(cls_prob[:, j] > np.float32(thresh))[0]
        if inds.size == 0:
            per_class.append(np.zeros((0, 5), np.float32))
            continue
        s = cls_prob[inds, j]
        order = np.argsort(-s, kind="stable")
        dets = np.concatenate([boxes[inds, j], s[:, None]], 1).astype(np.float32)[order]
        per_class.append(dets[nms(dets, nms_thresh)])
    if max_per_image > 0:
        scores = np.hstack([d[:, -1] for d in per_class[1:]])
        if len(scores) > max_per_image:
            th = np.sort(scores)[-max_per_image]
            per_class = [per_class[0]] + [d[np.where(d[:, -1] >= th)[0], :]
                                          for d in per_class[1:]]
    return per_class
