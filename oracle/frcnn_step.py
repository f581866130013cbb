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
from .daf_step import VGG16_CFG, _RoIAlignAvgCPU, _smooth_l1


class OracleFRCNN(nn.Module):
    def __init__(self, n_classes, scales=(8, 16, 32), ratios=(0.5, 1, 2), backbone="vgg16",
                 dropout=0.5, pre_post_train=(12000, 2000), pre_post_test=(6000, 300)):
        super().__init__()
        self.backbone = backbone
        self.rcnn_cfg = dict(orpn.DEFAULT_RCNN)
        A = len(scales) * len(ratios)
        if backbone == "vgg16":
            layers, cin = [], 3
            for v in VGG16_CFG:
                if v == "M":
                    layers.append(nn.MaxPool2d(2, 2))
                else:
                    layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                    cin = v
            self.RCNN_base = nn.Sequential(*layers)
            for i in range(10):
                for p in self.RCNN_base[i].parameters():
                    p.requires_grad = False
            self.RCNN_top = nn.Sequential(nn.Linear(25088, 4096), nn.ReLU(True), nn.Dropout(dropout),
                                          nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(dropout))
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
        x = F.relu(self.RCNN_rpn.RPN_Conv(base))
        score = self.RCNN_rpn.RPN_cls_score(x)
        B, C, H, W = score.shape
        sr = score.view(B, 2, C * H // 2, W)
        prob = F.softmax(sr, 1).view(B, C, H, W)
        bbox = self.RCNN_rpn.RPN_bbox_pred(x)
        pre, post = self.pre_post_train
        gt, info = gt.float(), info.float()  # the sampling ops see the reference's float32
        rois = orpn.proposal_layer(prob.detach().float().numpy(), bbox.detach().float().numpy(),
                                   info.numpy(),
                                   self.base_anchors, 16, pre, post, 0.7)
        if rois_override is not None:
            rois = rois_override
        lab, tgt, iw, ow = orpn.anchor_target(H, W, gt.numpy(), info.numpy(), self.base_anchors,
                                              16, rng)
        lab_t = torch.from_numpy(lab).view(-1)
        keep = lab_t != -1
        s2 = sr.permute(0, 2, 3, 1).contiguous().view(-1, 2)
        rpn_loss_cls = F.cross_entropy(s2[keep], lab_t[keep].long())
        rpn_loss_box = _smooth_l1(bbox, torch.from_numpy(tgt), torch.from_numpy(iw),
                                  torch.from_numpy(ow), sigma=3, dim=[1, 2, 3])
        r, rl, rt, riw, row = orpn.proposal_target(rois, gt.numpy(), rng, self.rcnn_cfg)
        rl = torch.from_numpy(rl).view(-1).long()
        pooled = _RoIAlignAvgCPU.apply(base, torch.from_numpy(r).view(-1, 5))
        fc7 = self._head_to_tail(pooled)
        bp = self.RCNN_bbox_pred(fc7).view(fc7.size(0), -1, 4)
        bp = torch.gather(bp, 1, rl.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        cls = self.RCNN_cls_score(fc7)
        rcnn_cls = F.cross_entropy(cls, rl)
        rcnn_box = _smooth_l1(bp, torch.from_numpy(rt).view(-1, 4),
                              torch.from_numpy(riw).view(-1, 4), torch.from_numpy(row).view(-1, 4))
        return dict(rpn_loss_cls=rpn_loss_cls, rpn_loss_box=rpn_loss_box, RCNN_loss_cls=rcnn_cls,
                    RCNN_loss_bbox=rcnn_box, rois=r, labels=rl)

    @torch.no_grad()
    def detect(self, im, info, rois):
        """Eval-mode head on given rois (faster_rcnn.py:70-113 with training False):
        (cls_prob (R, C), bbox_pred (R, 4C))."""
        base = self.RCNN_base(im)
        pooled = _RoIAlignAvgCPU.apply(base, torch.from_numpy(np.asarray(rois)).view(-1, 5))
        fc7 = self._head_to_tail(pooled)
        return F.softmax(self.RCNN_cls_score(fc7), 1), self.RCNN_bbox_pred(fc7)


def total_loss(o):
    return o["rpn_loss_cls"] + o["rpn_loss_box"] + o["RCNN_loss_cls"] + o["RCNN_loss_bbox"]
