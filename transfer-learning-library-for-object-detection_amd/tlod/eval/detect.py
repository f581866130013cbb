"""Test loop of the methods' *_test.py drivers (methods/DAF/DAF_test.py:239-354): the
detector in eval mode, per-class NMS and the per-image top-k, then VOC AP.

The per-class post-processing of one image — de-normalised deltas, bbox_transform_inv,
clip, / im_scale, score threshold, descending sort, NMS(TEST.NMS) for every class — is one
libtlod launch (tlod_detect_f32, one workgroup per class) instead of the reference's
Python loop with a host round trip per class.  The max_per_image cut (:323-333) and the
all_boxes bookkeeping stay on the host, as in the reference (its detections end there).
"""
import numpy as np
import torch

from .. import _lib
from ..config import cfg


def detect(rois, cls_prob, bbox_pred, im_info, class_agnostic=False, thresh=0.0, nms=None,
           return_boxes=False):
    """One image: rois (R, 5), cls_prob (R, C), bbox_pred (R, 4C | 4), im_info (3,) device
    tensors -> (dets (C, R, 5), counts (C,) int32[, boxes (R, C, 4)]) on the device."""
    _lib.require_cuda(rois, cls_prob, bbox_pred)
    rois = rois.detach().reshape(-1, 5).contiguous().float()
    cls_prob = cls_prob.detach().reshape(rois.shape[0], -1).contiguous().float()
    R, C = cls_prob.shape
    bbox_pred = bbox_pred.detach().reshape(R, -1).contiguous().float()
    assert bbox_pred.shape[1] == (4 if class_agnostic else 4 * C), bbox_pred.shape
    info = [float(v) for v in im_info.detach().reshape(-1).cpu().tolist()]
    stds = (ctypes_floats(cfg.TRAIN.BBOX_NORMALIZE_STDS)
            if cfg.TRAIN.BBOX_NORMALIZE_TARGETS_PRECOMPUTED else ctypes_floats((1, 1, 1, 1)))
    means = (ctypes_floats(cfg.TRAIN.BBOX_NORMALIZE_MEANS)
             if cfg.TRAIN.BBOX_NORMALIZE_TARGETS_PRECOMPUTED else ctypes_floats((0, 0, 0, 0)))
    dets = torch.empty((C, R, 5), dtype=torch.float32, device=rois.device)
    counts = torch.empty(C, dtype=torch.int32, device=rois.device)
    boxes = torch.zeros((R, C, 4), dtype=torch.float32, device=rois.device) if return_boxes \
        else None
    _lib.check(_lib.lib().tlod_detect_f32(
        _lib.ptr(rois), _lib.ptr(cls_prob), _lib.ptr(bbox_pred), R, C, int(class_agnostic), stds,
        means, info[0], info[1], info[2], float(thresh),
        float(cfg.TEST.NMS if nms is None else nms), _lib.ptr(dets), _lib.ptr(counts),
        _lib.ptr(boxes), _lib.stream_of(rois)), "detect")
    return (dets, counts, boxes) if return_boxes else (dets, counts)


def ctypes_floats(vals):
    import ctypes
    return (ctypes.c_float * 4)(*[float(v) for v in vals])


def limit_per_image(per_class, max_per_image):
    """DAF_test.py:323-333: keep the detections scoring >= the max_per_image-th best score
    over all classes.  per_class: list (index = class) of (n, 5) arrays."""
    if max_per_image <= 0:
        return per_class
    scores = np.hstack([d[:, -1] for d in per_class[1:]])
    if len(scores) > max_per_image:
        th = np.sort(scores)[-max_per_image]
        per_class = [per_class[0]] + [d[np.where(d[:, -1] >= th)[0], :] for d in per_class[1:]]
    return per_class


@torch.no_grad()
def im_detect(model, data, im_info, gt_boxes, num_boxes, max_per_image=100, thresh=0.0,
              class_agnostic=False):
    """The detections of one image (batch of 1): a list over classes of (n, 5) float32 numpy
    arrays (x1, y1, x2, y2, score) in original-image coordinates."""
    was = model.training
    model.eval()
    rois, cls_prob, bbox_pred = model(data, im_info, gt_boxes, num_boxes)[:3]
    model.train(was)
    dets, counts = detect(rois[0], cls_prob[0], bbox_pred[0], im_info.reshape(-1, 3)[0],
                          class_agnostic, thresh)
    d, n = dets.cpu().numpy(), counts.cpu().numpy()
    per_class = [np.zeros((0, 5), np.float32)] + [d[j, :n[j]] for j in range(1, d.shape[0])]
    return limit_per_image(per_class, max_per_image)


def eval_net(model, imdb, loader, output_dir, max_per_image=100, thresh=0.0,
             class_agnostic=False):
    """DAF_test.py:239-354 over a test roibatchLoader (training=False): all_boxes[class][image],
    then imdb.evaluate_detections -> {class: AP, "mAP": mean}."""
    all_boxes = [[[] for _ in range(imdb.num_images)] for _ in range(imdb.num_classes)]
    for i in range(imdb.num_images):
        item = loader[i]
        data, im_info, gt, num = (t.unsqueeze(0) for t in item[:4])
        per_class = im_detect(model, data, im_info, gt, num, max_per_image, thresh,
                              class_agnostic)
        for j in range(1, imdb.num_classes):
            all_boxes[j][i] = per_class[j]
    return imdb.evaluate_detections(all_boxes, output_dir), all_boxes
