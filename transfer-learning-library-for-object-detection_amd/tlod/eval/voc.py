"""PASCAL VOC detection AP — the metric of lib/datasets/voc_eval.py:15-211 (MIT), restated.

Same numbers as the reference's per-class evaluation (greedy matching of detections in
descending confidence to the highest-IoU ground truth of their image at IoU > ovthresh,
difficult objects neither counted nor penalised, a ground truth matched at most once;
VOC07 11-point or area-under-envelope AP), organised differently: annotations are parsed
into arrays once per image, detections are grouped per image and each image's IoU matrix
is computed in one broadcast, so the only Python loop left is the greedy assignment itself.
The reference's annotation pickle cache (voc_eval.py:110-128) is not kept.

Host-side numpy: it reads the comp4 result files the test driver writes
(lib/datasets/pascal_voc.py:284-298), off the device path.
"""
import xml.etree.ElementTree as ET

import numpy as np


def parse_rec(filename):
    """Objects of one VOC annotation file: dicts with name, pose, truncated, difficult and
    the 1-based integer bbox [xmin, ymin, xmax, ymax] (voc_eval.py:15-33)."""
    out = []
    for node in ET.parse(filename).findall("object"):
        box = node.find("bndbox")
        rec = {"name": node.find("name").text,
               "truncated": int(node.find("truncated").text),
               "difficult": int(node.find("difficult").text),
               "bbox": [int(box.find(tag).text) for tag in ("xmin", "ymin", "xmax", "ymax")]}
        pose = node.find("pose")
        if pose is not None:
            rec["pose"] = pose.text
        out.append(rec)
    return out


def voc_ap(rec, prec, use_07_metric=False):
    """AP from recall / precision curves (voc_eval.py:36-67): the mean of the maximum
    precision at recall >= 0, 0.1, ..., 1 (VOC07), or the area under the monotone
    precision envelope summed where recall changes."""
    rec = np.asarray(rec, dtype=np.float64)
    prec = np.asarray(prec, dtype=np.float64)
    if use_07_metric:
        total = 0.0
        for t in np.arange(0.0, 1.1, 0.1):  # accumulated in the reference's order
            hit = rec >= t
            total = total + (np.max(prec[hit]) if hit.any() else 0) / 11.0
        return total
    r = np.concatenate(([0.0], rec, [1.0]))
    envelope = np.maximum.accumulate(np.concatenate(([0.0], prec, [0.0]))[::-1])[::-1]
    steps = np.flatnonzero(r[1:] != r[:-1])
    return np.sum((r[steps + 1] - r[steps]) * envelope[steps + 1])


def _iou_matrix(det, gt):
    """IoU of every (detection, ground truth) pair with the reference's +1 pixel areas,
    elementwise the same float64 operations as voc_eval.py:165-180."""
    lo_x = np.maximum(gt[None, :, 0], det[:, None, 0])
    lo_y = np.maximum(gt[None, :, 1], det[:, None, 1])
    hi_x = np.minimum(gt[None, :, 2], det[:, None, 2])
    hi_y = np.minimum(gt[None, :, 3], det[:, None, 3])
    inter = np.maximum(hi_x - lo_x + 1.0, 0.0) * np.maximum(hi_y - lo_y + 1.0, 0.0)
    det_area = (det[:, 2] - det[:, 0] + 1.0) * (det[:, 3] - det[:, 1] + 1.0)
    gt_area = (gt[:, 2] - gt[:, 0] + 1.0) * (gt[:, 3] - gt[:, 1] + 1.0)
    return inter / (det_area[:, None] + gt_area[None, :] - inter)


def _read_detections(detpath):
    """(image ids, confidences, boxes) of a comp4 results file: "<image> <score> <x1> <y1>
    <x2> <y2>" per line."""
    with open(detpath) as f:
        fields = [line.strip().split(" ") for line in f]
    ids = [row[0] for row in fields]
    scores = np.array([float(row[1]) for row in fields])
    boxes = np.array([[float(v) for v in row[2:]] for row in fields], dtype=np.float64).reshape(-1, 4)
    return ids, scores, boxes


def voc_eval(detpath, annopath, imagesetfile, classname, ovthresh=0.5, use_07_metric=False):
    """(rec, prec, ap) of one class (voc_eval.py:70-211).  detpath: the class's results
    file; annopath: a format string of the annotation path per image name."""
    with open(imagesetfile) as f:
        names = [line.strip() for line in f]
    gt_box, gt_hard = {}, {}
    npos = 0
    for name in names:
        objs = [o for o in parse_rec(annopath.format(name)) if o["name"] == classname]
        gt_box[name] = np.array([o["bbox"] for o in objs], dtype=np.float64).reshape(-1, 4)
        gt_hard[name] = np.array([bool(o["difficult"]) for o in objs], dtype=bool)
        npos += int((~gt_hard[name]).sum())

    ids, scores, boxes = _read_detections(detpath)
    nd = len(ids)
    tp = np.zeros(nd)
    fp = np.zeros(nd)
    if nd:
        order = np.argsort(-scores)  # the reference's call: the same order for ties
        ranked_ids = [ids[k] for k in order]
        ranked_boxes = boxes[order].astype(float)
        by_image = {}
        for rank, name in enumerate(ranked_ids):
            by_image.setdefault(name, []).append(rank)
        for name, ranks in by_image.items():
            ranks = np.array(ranks)
            gts = gt_box[name]
            if gts.shape[0] == 0:  # no ground truth of the class in this image
                fp[ranks] = 1.0
                continue
            iou = _iou_matrix(ranked_boxes[ranks], gts)
            best = iou.argmax(axis=1)
            best_iou = iou[np.arange(len(ranks)), best]
            taken = np.zeros(gts.shape[0], dtype=bool)
            for rank, j, ov in zip(ranks, best, best_iou):  # greedy, in confidence order
                if not ov > ovthresh:
                    fp[rank] = 1.0
                elif gt_hard[name][j]:
                    continue
                elif taken[j]:
                    fp[rank] = 1.0
                else:
                    tp[rank] = 1.0
                    taken[j] = True
    ctp = np.cumsum(tp)
    cfp = np.cumsum(fp)
    rec = ctp / float(npos)
    prec = ctp / np.maximum(ctp + cfp, np.finfo(np.float64).eps)
    return rec, prec, voc_ap(rec, prec, use_07_metric)
