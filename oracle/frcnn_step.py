"""Oracle: the source-only Faster R-CNN training step on the CPU (TEST INFRASTRUCTURE ONLY).

Restates lib/model/faster_rcnn/faster_rcnn.py:39-115 with lib/model/faster_rcnn/vgg16.py
(or the ResNet101 parts of oracle.resnet) and the loss sum of
methods/faster_rcnn/faster_rcnn_train.py:326-327, in torch-CPU fp32 (conv / linear /
softmax: the third-party arithmetic, "parity unpinned" at that boundary) plus the numpy
restatements of the reference's own ops (oracle.rpn / oracle.roi).  Module names follow
the reference's state_dict keys, so the device model's weights load strictly.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import rpn as orpn
from .daf_step import SiteReLU, _np, _RoIAlignAvgCPU, _smooth_l1, _t, forced_relu, vgg16_features


class OracleFRCNN(nn.Module):
    def __init__(self, n_classes, scales=(8, 16, 32), ratios=(0.5, 1, 2), backbone="vgg16",
                 dropout=0.5, pre_post_train=(12000, 2000), pre_post_test=(6000, 300)):
        super().__init__()
        self.backbone = backbone
        self.rcnn_cfg = dict(orpn.DEFAULT_RCNN)
        A = len(scales) * len(ratios)
        self.forced = {}  # site -> forced masks / pool indices (oracle.daf_step.forced_relu)
        if backbone == "vgg16":
            self.RCNN_base = vgg16_features(self.forced)
            for i in range(10):
                for p in self.RCNN_base[i].parameters():
                    p.requires_grad = False
            self.RCNN_top = nn.Sequential(nn.Linear(25088, 4096), SiteReLU(self.forced, "fc6"),
                                          nn.Dropout(dropout), nn.Linear(4096, 4096),
                                          SiteReLU(self.forced, "fc7"), nn.Dropout(dropout))
            din, dfeat = 512, 4096
        else:
            from .resnet import resnet101_parts
            self.RCNN_base, self.RCNN_top = resnet101_parts()
            self.rcnn_cfg["batch"] = 128
            din, dfeat = 1024, 2048
        self.RCNN_cls_score = nn.Linear(dfeat, n_classes)
        self.RCNN_bbox_pred = nn.Linear(dfeat, 4 * n_classes)
        rpn = nn.Module()
        rpn.RPN_Conv = nn.Conv2d(din, 512, 3, padding=1)
        rpn.RPN_cls_score = nn.Conv2d(512, 2 * A, 1)
        rpn.RPN_bbox_pred = nn.Conv2d(512, 4 * A, 1)
        self.RCNN_rpn = rpn
        self.base_anchors = orpn.make_base_anchors(scales, ratios)
        self.pre_post_train, self.pre_post_test = pre_post_train, pre_post_test

    def train(self, mode=True):
        super().train(mode)
        if self.backbone == "res101":
            from .resnet import bn_eval
            bn_eval(self)
        return self

    def _head_to_tail(self, pooled):
        if self.backbone == "res101":
            return self.RCNN_top(pooled).mean(3).mean(2)
        return self.RCNN_top(pooled.view(pooled.size(0), -1))

    def forward(self, im, info, gt, rng, rois_override=None):
        """Training-mode losses (faster_rcnn.py:39-115).  rois_override: the device run's
        proposals (the score sort of near-tied random-init scores is order-sensitive)."""
        base = self.RCNN_base(im)
        x = forced_relu(self.forced, "rpn", self.RCNN_rpn.RPN_Conv(base))
        score = self.RCNN_rpn.RPN_cls_score(x)
        B, C, H, W = score.shape
        sr = score.view(B, 2, C * H // 2, W)
        prob = F.softmax(sr, 1).view(B, C, H, W)
        bbox = self.RCNN_rpn.RPN_bbox_pred(x)
        pre, post = self.pre_post_train
        gt, info = gt.float(), info.float()  # the sampling ops see the reference's float32
        rois = orpn.proposal_layer(_np(prob.float()), _np(bbox.float()),
                                   _np(info),
                                   self.base_anchors, 16, pre, post, 0.7)
        if rois_override is not None:
            rois = rois_override
        lab, tgt, iw, ow = orpn.anchor_target(H, W, _np(gt), _np(info), self.base_anchors,
                                              16, rng)
        lab_t = _t(lab, bbox).view(-1)
        keep = lab_t != -1
        s2 = sr.permute(0, 2, 3, 1).contiguous().view(-1, 2)
        rpn_loss_cls = F.cross_entropy(s2[keep], lab_t[keep].long())
        rpn_loss_box = _smooth_l1(bbox, _t(tgt, bbox), _t(iw, bbox),
                                  _t(ow, bbox), sigma=3, dim=[1, 2, 3])
        r, rl, rt, riw, row = orpn.proposal_target(rois, _np(gt), rng, self.rcnn_cfg)
        rl = _t(rl, bbox).view(-1).long()
        pooled = _RoIAlignAvgCPU.apply(base, _t(r, base).view(-1, 5))
        fc7 = self._head_to_tail(pooled)
        bp = self.RCNN_bbox_pred(fc7).view(fc7.size(0), -1, 4)
        bp = torch.gather(bp, 1, rl.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        cls = self.RCNN_cls_score(fc7)
        rcnn_cls = F.cross_entropy(cls, rl)
        rcnn_box = _smooth_l1(bp, _t(rt, bp).view(-1, 4),
                              _t(riw, bp).view(-1, 4), _t(row, bp).view(-1, 4))
        return dict(rpn_loss_cls=rpn_loss_cls, rpn_loss_box=rpn_loss_box, RCNN_loss_cls=rcnn_cls,
                    RCNN_loss_bbox=rcnn_box, rois=r, labels=rl)

    @torch.no_grad()
    def detect(self, im, info, rois):
        """Eval-mode head on given rois (faster_rcnn.py:70-113 with training False):
        (cls_prob (R, C), bbox_pred (R, 4C))."""
        base = self.RCNN_base(im)
        pooled = _RoIAlignAvgCPU.apply(base, _t(np.asarray(rois), base).view(-1, 5))
        fc7 = self._head_to_tail(pooled)
        return F.softmax(self.RCNN_cls_score(fc7), 1), self.RCNN_bbox_pred(fc7)


def total_loss(o):
    return o["rpn_loss_cls"] + o["rpn_loss_box"] + o["RCNN_loss_cls"] + o["RCNN_loss_bbox"]
