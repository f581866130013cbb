"""Oracle: the ATF VGG16 training step on the CPU (test infrastructure only).

A literal restatement of lib/ATF/faster_rcnn.py:108-363 + methods/ATF/ATF_train.py:405-408:
separate passes for every branch and image (conv3_t recomputes the shared frozen conv1/2
on the source image, the RPN runs twice in train mode, the target RPN runs in eval mode
with TEST post-NMS top-N = 2000), torch-CPU fp32 conv/linear ("parity unpinned" at that
boundary, as for DAF) and the numpy restatements of the reference's own ops.
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import rpn as orpn
from .daf_step import (CFG, OracleDAF, SitePool, SiteReLU, _RoIAlignAvgCPU, _np, _smooth_l1, _t,
                       forced_relu)


class OracleATF(OracleDAF):
    def __init__(self, n_classes=9, dropout=0.5, backbone="vgg16"):
        super().__init__(n_classes, dropout, backbone)
        shared = self.splits[0]
        layers = list(self.RCNN_base)
        self.RCNN_base_t = nn.Sequential(*(layers[:shared] + [copy.deepcopy(m) for m in layers[shared:]]))
        # the t branch's activation sites: base_t.* on the model's own forced dict
        for i in range(shared, len(layers)):
            for mod in self.RCNN_base_t[i].modules():
                if isinstance(mod, (SiteReLU, SitePool)):
                    mod.forced, mod.site = self.forced, mod.site.replace("base.", "base_t.", 1)
        if backbone == "res101":
            from .resnet import name_sites
            name_sites(self.RCNN_base_t[shared:], self.forced, "base_t")
            for mod in self.RCNN_base_t[shared:].modules():  # index i counts from `shared`
                if getattr(mod, "site", None) and mod.site.startswith("base_t."):
                    i, rest = mod.site[len("base_t."):].split(".", 1)
                    mod.site = f"base_t.{int(i) + shared}.{rest}"
        for name, dim in (("RCNN_imageDA_3", 256), ("RCNN_imageDA_4", 512)):
            m = nn.Module()
            m.Conv1 = nn.Conv2d(dim, 512, 1, bias=False)
            m.Conv2 = nn.Conv2d(512, 2, 1, bias=False)
            setattr(self, name, m)

    def _da(self, m, feat, site):
        from .daf_step import _GRL
        return m.Conv2(forced_relu(self.forced, site, m.Conv1(_GRL.apply(feat, 0.1))))

    @staticmethod
    def _nll(score, label):
        lab = torch.full((score.shape[0], *score.shape[2:]), label, dtype=torch.long,
                         device=score.device)
        return F.nll_loss(F.log_softmax(score, 1), lab, ignore_index=-1)

    def _rpn_train(self, feat, gt, info, rng, rois_override):
        c = CFG
        score, sr, prob, bbox = self._rpn(feat)
        gt, info = gt.float(), info.float()  # the sampling ops see the reference's float32
        rois = orpn.proposal_layer(_np(prob.float()), _np(bbox.float()), _np(info),
                                   self.base_anchors, c["stride"], c["pre_train"], c["post_train"],
                                   c["nms"])
        props = rois
        if rois_override is not None:
            rois = rois_override
        H, W = score.shape[2:]
        lab, tgt, iw, ow = orpn.anchor_target(H, W, _np(gt), _np(info), self.base_anchors,
                                              c["stride"], rng)
        lab_t = _t(lab, bbox).view(-1)
        keep = lab_t != -1
        s2 = sr.permute(0, 2, 3, 1).contiguous().view(-1, 2)
        loss_cls = F.cross_entropy(s2[keep], lab_t[keep].long())
        loss_box = _smooth_l1(bbox, _t(tgt, bbox), _t(iw, bbox), _t(ow, bbox), sigma=3,
                              dim=[1, 2, 3])
        return rois, props, loss_cls, loss_box

    def _det_losses(self, fc7, rl, rt, riw, row):
        bp = self.RCNN_bbox_pred(fc7).view(fc7.size(0), -1, 4)
        bp = torch.gather(bp, 1, rl.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        cls = self.RCNN_cls_score(fc7)
        return F.cross_entropy(cls, rl), _smooth_l1(bp, rt, riw, row)

    def forward(self, batch, rng, rois_override=None):
        """rois_override: (s-branch, t-branch, target) proposal arrays from the device run."""
        (im, info, gt, num, need, t_im, t_info, t_gt, t_num, t_need) = batch
        c = CFG
        ov = rois_override or (None, None, None)
        _, e3, e4 = self.splits
        base = self.RCNN_base(im)
        c3_t = self.RCNN_base_t[:e3](im)
        c4_t = self.RCNN_base_t[e3:e4](c3_t)
        base_t = self.RCNN_base_t[e4:](c4_t)
        rois_domain, props_s, l1c, l1b = self._rpn_train(base, gt, info, rng, ov[0])
        rois_domain_t, props_st, l2c, l2b = self._rpn_train(base_t, gt, info, rng, ov[1])

        def sample(r):
            r, rl, rt, riw, row = orpn.proposal_target(r, _np(gt.float()), rng, self.rcnn_cfg)
            return (r, _t(rl, base).view(-1).long(), _t(rt, base).view(-1, 4),
                    _t(riw, base).view(-1, 4), _t(row, base).view(-1, 4))
        r_s, rl_s, rt_s, riw_s, row_s = sample(rois_domain)
        r_t, rl_t, rt_t, riw_t, row_t = sample(rois_domain_t)

        def head(feat, rois):
            p = _RoIAlignAvgCPU.apply(feat, _t(rois, feat).view(-1, 5))
            return self._head_to_tail(p)
        fc7_s, fc7_t, fc7_dt = head(base, r_s), head(base_t, r_t), head(base_t, rois_domain_t)
        cls_s, box_s = self._det_losses(fc7_s, rl_s, rt_s, riw_s, row_s)
        cls_t, box_t = self._det_losses(fc7_t, rl_t, rt_t, riw_t, row_t)

        t_c3, t_c4, t_base = self._backbone(t_im)
        _, _, t_prob, t_bbox = self._rpn(t_base)
        t_rois = orpn.proposal_layer(_np(t_prob.float()), _np(t_bbox.float()),
                                     _np(t_info.float()), self.base_anchors, c["stride"],
                                     c["pre_test"], rois_domain.shape[1], c["nms"])
        props_t = t_rois
        if ov[2] is not None:
            t_rois = ov[2]
        fc7_tgt = head(t_base, t_rois)

        da = self._nll(self._da(self.RCNN_imageDA_3, c3_t, "ida3"), 1) + \
            self._nll(self._da(self.RCNN_imageDA_4, c4_t, "ida4"), 1) + \
            self._nll(self._image_da(base_t), 1)
        t_da = self._nll(self._da(self.RCNN_imageDA_3, t_c3, "ida3"), 0) + \
            self._nll(self._da(self.RCNN_imageDA_4, t_c4, "ida4"), 0) + \
            self._nll(self._image_da(t_base), 0)
        ins = self._instance_da(fc7_dt)
        y = torch.zeros_like(ins)
        y[:256] = 1.0  # ATF InstanceLabelResizeLayer (lib/ATF/LabelResizeLayer.py:50-60)
        t_ins = self._instance_da(fc7_tgt)
        return dict(rpn_loss_cls=l1c + l2c, rpn_loss_box=l1b + l2b, RCNN_loss_cls=cls_s + cls_t,
                    RCNN_loss_bbox=box_s + box_t, DA_img_loss_cls=da, tgt_DA_img_loss_cls=t_da,
                    DA_ins_loss_cls=F.binary_cross_entropy(ins, y),
                    tgt_DA_ins_loss_cls=F.binary_cross_entropy(t_ins, torch.zeros_like(t_ins)),
                    rois=r_t, props_s=props_s, props_st=props_st, props_t=props_t)


def total_loss(o, lamda=0.1):
    """methods/ATF/ATF_train.py:405-408."""
    return (o["rpn_loss_cls"] + o["rpn_loss_box"] + o["RCNN_loss_cls"] + o["RCNN_loss_bbox"]
            + lamda * (7 * o["DA_img_loss_cls"] + o["DA_ins_loss_cls"]
                       + 7 * o["tgt_DA_img_loss_cls"] + o["tgt_DA_ins_loss_cls"]))
