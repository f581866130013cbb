"""PASCAL VOC detection AP (lib/datasets/voc_eval.py:15-211), the reference's Python eval.

Host-side numpy, as in the reference (it reads the comp4 results files the test driver
wrote, lib/datasets/pascal_voc.py:284-298).  The annotation pickle cache of the reference
(voc_eval.py:110-128) is not kept: annotations are parsed each call.
"""
import xml.etree.ElementTree as ET

import numpy as np


def parse_rec(filename):
    """voc_eval.py:15-33."""
    tree = ET.parse(filename)
    objects = []
    for obj in tree.findall("object"):
        o = {"name": obj.find("name").text}
        if obj.find("pose") is not None:
            o["pose"] = obj.find("pose").text
        o["truncated"] = int(obj.find("truncated").text)
        o["difficult"] = int(obj.find("difficult").text)
        bbox = obj.find("bndbox")
        o["bbox"] = [int(bbox.find(k).text) for k in ("xmin", "ymin", "xmax", "ymax")]
        objects.append(o)
    return objects


def voc_ap(rec, prec, use_07_metric=False):
    """voc_eval.py:36-67: VOC07 11-point AP, or the area under the precision envelope."""
    if use_07_metric:
        ap = 0.0
        for t in np.arange(0.0, 1.1, 0.1):
            p = 0 if np.sum(rec >= t) == 0 else np.max(prec[rec >= t])
            ap = ap + p / 11.0
        return ap
    mrec = np.concatenate(([0.0], rec, [1.0]))
    mpre = np.concatenate(([0.0], prec, [0.0]))
    for i in range(mpre.size - 1, 0, -1):
        mpre[i - 1] = np.maximum(mpre[i - 1], mpre[i])
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1])


def voc_eval(detpath, annopath, imagesetfile, classname, ovthresh=0.5, use_07_metric=False):
    """voc_eval.py:70-211 -> (rec, prec, ap) for one class.  detpath: the class's results
    file ("<image> <score> <x1> <y1> <x2> <y2>" per line, 1-based); annopath: a format
    string of the annotation path per image name."""
    with open(imagesetfile) as f:
        imagenames = [x.strip() for x in f.readlines()]
    recs = {name: parse_rec(annopath.format(name)) for name in imagenames}
    class_recs = {}
    npos = 0
    for name in imagenames:
        R = [o for o in recs[name] if o["name"] == classname]
        bbox = np.array([x["bbox"] for x in R])
        difficult = np.array([x["difficult"] for x in R]).astype(bool)
        npos = npos + sum(~difficult)
        class_recs[name] = {"bbox": bbox, "difficult": difficult, "det": [False] * len(R)}
    with open(detpath) as f:
        lines = f.readlines()
    splitlines = [x.strip().split(" ") for x in lines]
    image_ids = [x[0] for x in splitlines]
    confidence = np.array([float(x[1]) for x in splitlines])
    BB = np.array([[float(z) for z in x[2:]] for x in splitlines])
    nd = len(image_ids)
    tp = np.zeros(nd)
    fp = np.zeros(nd)
    if BB.shape[0] > 0:
        sorted_ind = np.argsort(-confidence)
        BB = BB[sorted_ind, :]
        image_ids = [image_ids[x] for x in sorted_ind]
        for d in range(nd):
            R = class_recs[image_ids[d]]
            bb = BB[d, :].astype(float)
            ovmax = -np.inf
            BBGT = R["bbox"].astype(float)
            if BBGT.size > 0:
                ixmin = np.maximum(BBGT[:, 0], bb[0])
                iymin = np.maximum(BBGT[:, 1], bb[1])
                ixmax = np.minimum(BBGT[:, 2], bb[2])
                iymax = np.minimum(BBGT[:, 3], bb[3])
                iw = np.maximum(ixmax - ixmin + 1.0, 0.0)
                ih = np.maximum(iymax - iymin + 1.0, 0.0)
                inters = iw * ih
                uni = ((bb[2] - bb[0] + 1.0) * (bb[3] - bb[1] + 1.0)
                       + (BBGT[:, 2] - BBGT[:, 0] + 1.0) * (BBGT[:, 3] - BBGT[:, 1] + 1.0) - inters)
                overlaps = inters / uni
                ovmax = np.max(overlaps)
                jmax = np.argmax(overlaps)
            if ovmax > ovthresh:
                if not R["difficult"][jmax]:
                    if not R["det"][jmax]:
                        tp[d] = 1.0
                        R["det"][jmax] = 1
                    else:
                        fp[d] = 1.0
            else:
                fp[d] = 1.0
    fp = np.cumsum(fp)
    tp = np.cumsum(tp)
    rec = tp / float(npos)
    prec = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
    return rec, prec, voc_ap(rec, prec, use_07_metric)
