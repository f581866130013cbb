"""Oracle: the DAF VGG16 training step on the CPU (test infrastructure + bench.py's
cpu_baseline leg only).

A restatement of lib/DAF/faster_rcnn.py:45-224 + methods/DAF/DAF_train.py:384-408 in
plain torch-CPU fp32 (conv/linear/pool/softmax — the third-party arithmetic the reference
gets from PyTorch, "parity unpinned" at that boundary) with the numpy restatements of the
reference's own ops (oracle.rpn / oracle.roi / oracle.nms).  Module names mirror the
reference's state_dict keys so weights can be copied from the GPU model.
"""
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import roi as oroi
from . import rpn as orpn

VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512]
CFG = dict(pre_train=12000, post_train=2000, pre_test=6000, post_test=300, nms=0.7,
           scales=(4, 8, 16, 32), ratios=(0.5, 1, 2), stride=16, pool=7, lamda=0.1)


def _np(t):
    return t.detach().cpu().numpy()


def _t(a, like):
    """numpy result of a restated op -> a tensor next to ``like`` (the oracle's torch parts
    may run on the GPU: the reference's own fp32 arithmetic on this hardware)."""
    return torch.from_numpy(np.ascontiguousarray(a)).to(like.device)


class _RoIAlignAvgCPU(torch.autograd.Function):
    """float32 features: the CUDA kernels' arithmetic; float64 features (the exact-arithmetic
    reference of the gradient bars): the same sample geometry in double."""

    @staticmethod
    def forward(ctx, feat, rois):
        f = _np(feat)
        r = _np(rois.float())
        ctx.meta = (r, f.shape, f.dtype, feat.device)
        if f.dtype == np.float64:
            return _t(oroi.roi_align_avg_fwd64(f, r, CFG["pool"], CFG["pool"], 1 / 16), feat)
        return _t(oroi.roi_align_avg_fwd(f, r, CFG["pool"], CFG["pool"], 1 / 16), feat)

    @staticmethod
    def backward(ctx, g):
        r, (B, C, H, W), dt, _ = ctx.meta
        if dt == np.float64:
            return _t(oroi.roi_align_avg_bwd64(_np(g), r, B, C, H, W, 1 / 16), g), None
        return _t(oroi.roi_align_avg_bwd(_np(g), r, B, C, H, W, 1 / 16), g), None


def forced_relu(forced, site, x):
    """ReLU, or — when ``forced`` holds masks for ``site`` — x * mask with the next mask of
    that site: the fp64 gradient reference evaluated in the device's activation pattern
    (a pre-activation within rounding of 0 may land on either side in two fp32 runs; the
    gradient of the same piecewise-linear function needs the same side)."""
    if forced and forced.get("__record__") is not None:  # record this run's own masks
        forced["__record__"].setdefault(site, []).append((x > 0).detach())
    lst = forced.get(site) if forced else None
    if lst:
        return x * lst.pop(0).to(device=x.device, dtype=x.dtype)
    return F.relu(x)


class SiteReLU(nn.Module):
    def __init__(self, forced, site):
        super().__init__()
        self.forced, self.site = forced, site

    def forward(self, x):
        return forced_relu(self.forced, self.site, x)


class SitePool(nn.Module):
    """MaxPool2d(2, 2), or a gather at forced argmax indices (max_pool2d return_indices
    layout) for the same reason."""

    def __init__(self, forced, site):
        super().__init__()
        self.forced, self.site = forced, site

    def forward(self, x):
        if self.forced and self.forced.get("__record__") is not None:
            self.forced["__record__"].setdefault(self.site, []).append(
                F.max_pool2d(x.detach(), 2, 2, return_indices=True)[1])
        lst = self.forced.get(self.site) if self.forced else None
        if not lst:
            return F.max_pool2d(x, 2, 2)
        idx = lst.pop(0).to(x.device)
        B, C, H, W = x.shape
        return x.reshape(B, C, H * W).gather(2, idx.reshape(B, C, -1)).reshape(idx.shape)


def vgg16_features(forced):
    """torchvision vgg16().features[:-1] with named activation / pool sites."""
    layers, cin = [], 3
    for v in VGG16_CFG:
        if v == "M":
            layers.append(SitePool(forced, f"base.{len(layers)}"))
        else:
            layers += [nn.Conv2d(cin, v, 3, padding=1), SiteReLU(forced, f"base.{len(layers) + 1}")]
            cin = v
    return nn.Sequential(*layers)


class _GRL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, alpha):
        ctx.alpha = alpha
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.neg() * ctx.alpha, None


def _smooth_l1(pred, target, iw, ow, sigma=1.0, dim=(1,)):
    s2 = sigma ** 2
    d = iw * (pred - target)
    a = d.abs()
    sign = (a < 1.0 / s2).float()
    loss = ow * (d.pow(2) * (s2 / 2.0) * sign + (a - 0.5 / s2) * (1.0 - sign))
    for i in sorted(dim, reverse=True):
        loss = loss.sum(i)
    return loss.mean()


class OracleDAF(nn.Module):
    """backbone "vgg16" (lib/DAF/vgg16.py) or "res101" (lib/DAF/resnet.py, oracle.resnet;
    RoI batch 128 from cfgs/res101.yml, instance head on the 2048-d features)."""

    def __init__(self, n_classes=9, dropout=0.5, backbone="vgg16"):
        super().__init__()
        self.backbone = backbone
        self.rcnn_cfg = dict(orpn.DEFAULT_RCNN)
        self.forced = {}  # site -> masks / pool indices to use instead of recomputing them
        if backbone == "vgg16":
            self.RCNN_base = vgg16_features(self.forced)
            for i in range(10):
                for p in self.RCNN_base[i].parameters():
                    p.requires_grad = False
            self.RCNN_top = nn.Sequential(nn.Linear(25088, 4096), SiteReLU(self.forced, "fc6"),
                                          nn.Dropout(dropout), nn.Linear(4096, 4096),
                                          SiteReLU(self.forced, "fc7"), nn.Dropout(dropout))
            din, dfeat = 512, 4096
            self.splits = (10, 16, 23)  # shared frozen prefix, conv3 end, conv4 end
        else:
            from .resnet import name_sites, resnet101_parts
            self.RCNN_base, self.RCNN_top = resnet101_parts()
            name_sites(self.RCNN_base, self.forced, "base")
            name_sites(self.RCNN_top, self.forced, "top")
            self.rcnn_cfg["batch"] = 128
            din, dfeat = 1024, 2048
            self.splits = (5, 5, 6)  # conv1..layer1 | layer2 | layer3
        self.RCNN_cls_score = nn.Linear(dfeat, n_classes)
        self.RCNN_bbox_pred = nn.Linear(dfeat, 4 * n_classes)
        rpn = nn.Module()
        rpn.RPN_Conv = nn.Conv2d(din, 512, 3, padding=1)
        rpn.RPN_cls_score = nn.Conv2d(512, 24, 1)
        rpn.RPN_bbox_pred = nn.Conv2d(512, 48, 1)
        self.RCNN_rpn = rpn
        ida = nn.Module()
        ida.Conv1 = nn.Conv2d(din, 512, 1, bias=False)
        ida.Conv2 = nn.Conv2d(512, 2, 1, bias=False)
        self.RCNN_imageDA = ida
        ins = nn.Module()
        ins.dc_ip1, ins.dc_ip2, ins.clssifer = nn.Linear(dfeat, 1024), nn.Linear(1024, 1024), nn.Linear(1024, 1)
        self.RCNN_instanceDA = ins
        self.dropout = dropout
        self.base_anchors = orpn.make_base_anchors(CFG["scales"], CFG["ratios"])

    def _rpn(self, feat):
        x = forced_relu(self.forced, "rpn", self.RCNN_rpn.RPN_Conv(feat))
        score = self.RCNN_rpn.RPN_cls_score(x)
        B, C, H, W = score.shape
        sr = score.view(B, 2, C * H // 2, W)
        prob = F.softmax(sr, 1).view(B, C, H, W)
        return score, sr, prob, self.RCNN_rpn.RPN_bbox_pred(x)

    def _image_da(self, feat):
        x = _GRL.apply(feat, 0.1)
        return self.RCNN_imageDA.Conv2(forced_relu(self.forced, "ida", self.RCNN_imageDA.Conv1(x)))

    def _instance_da(self, x):
        m = self.RCNN_instanceDA
        x = _GRL.apply(x, 0.1)
        x = F.dropout(forced_relu(self.forced, "ip1", m.dc_ip1(x)), self.dropout, self.training)
        x = F.dropout(forced_relu(self.forced, "ip2", m.dc_ip2(x)), self.dropout, self.training)
        return torch.sigmoid(m.clssifer(x))

    def train(self, mode=True):
        super().train(mode)
        if self.backbone == "res101":  # resnet.py:269-284
            from .resnet import bn_eval
            bn_eval(self)
        return self

    def _head_to_tail(self, pooled):
        if self.backbone == "res101":
            return self.RCNN_top(pooled).mean(3).mean(2)  # resnet.py:286-288
        return self.RCNN_top(pooled.view(pooled.size(0), -1))

    def _backbone(self, im):
        """RCNN_base in the three pieces MAF / ATF tap (lib/MAF/vgg16.py:84-86): conv3 =
        features[:16], conv34 = [16:23], conv45 = [23:-1]; ResNet101: conv1..layer1 |
        layer2 | layer3 (lib/ATF/resnet.py:238-241)."""
        _, e3, e4 = self.splits
        c3 = self.RCNN_base[:e3](im)
        c4 = self.RCNN_base[e3:e4](c3)
        return c3, c4, self.RCNN_base[e4:](c4)

    def _detect(self, batch, rng, rois_override=None):
        """Everything but the DA heads (lib/DAF/faster_rcnn.py:45-175).  rois_override:
        (source proposals (1,2000,5), target proposals (1,300,5)) taken from the device
        run, so float-order differences in the score sort cannot fork the sampled RoIs
        between the two implementations."""
        (im, info, gt, num, need, t_im, t_info, t_gt, t_num, t_need) = batch
        c = CFG
        c3, c4, base = self._backbone(im)
        score, sr, prob, bbox = self._rpn(base)
        gt, info = gt.float(), info.float()  # the sampling ops see the reference's float32
        rois = orpn.proposal_layer(_np(prob.float()), _np(bbox.float()), _np(info),
                                   self.base_anchors, c["stride"], c["pre_train"], c["post_train"],
                                   c["nms"])
        props = rois
        if rois_override is not None:
            rois = rois_override[0]
        H, W = score.shape[2:]
        lab, tgt, iw, ow = orpn.anchor_target(H, W, _np(gt), _np(info), self.base_anchors,
                                              c["stride"], rng)
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
        rcnn_box = _smooth_l1(bp, _t(rt, bp).view(-1, 4), _t(riw, bp).view(-1, 4),
                              _t(row, bp).view(-1, 4))
        # target image: RPN in eval mode (TEST proposals)
        t_c3, t_c4, t_base = self._backbone(t_im)
        _, _, t_prob, t_bbox = self._rpn(t_base)
        t_rois = orpn.proposal_layer(_np(t_prob.float()), _np(t_bbox.float()),
                                     _np(t_info.float()), self.base_anchors, c["stride"], c["pre_test"],
                                     c["post_test"], c["nms"])
        t_props = t_rois
        if rois_override is not None:
            t_rois = rois_override[1]
        t_pooled = _RoIAlignAvgCPU.apply(t_base, _t(t_rois, t_base).view(-1, 5))
        t_fc7 = self._head_to_tail(t_pooled)
        return dict(rpn_loss_cls=rpn_loss_cls, rpn_loss_box=rpn_loss_box, RCNN_loss_cls=rcnn_cls,
                    RCNN_loss_bbox=rcnn_box, rois=r, props=props, t_props=t_props, c3=c3, c4=c4,
                    base=base, fc7=fc7, cls=cls,
                    t_c3=t_c3, t_c4=t_c4, t_base=t_base, t_fc7=t_fc7)

    def forward(self, batch, rng, rois_override=None):
        d = self._detect(batch, rng, rois_override)
        base, fc7, t_base, t_fc7 = d["base"], d["fc7"], d["t_base"], d["t_fc7"]
        # DA (faster_rcnn.py:181-220)
        bs = self._image_da(base)
        da_img = F.nll_loss(F.log_softmax(bs, 1), torch.ones(bs.shape[0], *bs.shape[2:], dtype=torch.long,
                                                             device=bs.device))
        ins = self._instance_da(fc7)
        da_ins = F.binary_cross_entropy(ins, torch.ones_like(ins))
        cst = F.softmax(bs, 1)[:, 1].mean().detach()
        da_cst = ((ins - cst) ** 2).sum()
        tbs = self._image_da(t_base)
        t_da_img = F.nll_loss(F.log_softmax(tbs, 1), torch.zeros(tbs.shape[0], *tbs.shape[2:],
                                                                dtype=torch.long, device=tbs.device))
        t_ins = self._instance_da(t_fc7)
        y = torch.ones_like(t_ins)
        y[:256] = 0  # InstanceLabelResizeLayer quirk (LabelResizeLayer.py:48-55)
        t_da_ins = F.binary_cross_entropy(t_ins, y)
        t_cst = F.softmax(tbs, 1)[:, 0].mean().detach()
        t_da_cst = ((t_ins - t_cst) ** 2).sum()
        return dict(rpn_loss_cls=d["rpn_loss_cls"], rpn_loss_box=d["rpn_loss_box"],
                    RCNN_loss_cls=d["RCNN_loss_cls"], RCNN_loss_bbox=d["RCNN_loss_bbox"],
                    DA_img_loss_cls=da_img, DA_ins_loss_cls=da_ins,
                    tgt_DA_img_loss_cls=t_da_img, tgt_DA_ins_loss_cls=t_da_ins, DA_cst_loss=da_cst,
                    tgt_DA_cst_loss=t_da_cst, rois=d["rois"])


def total_loss(o, lamda=0.1):
    return (o["rpn_loss_cls"] + o["rpn_loss_box"] + o["RCNN_loss_cls"] + o["RCNN_loss_bbox"]
            + lamda * (o["DA_img_loss_cls"] + o["DA_ins_loss_cls"] + o["tgt_DA_img_loss_cls"]
                       + o["tgt_DA_ins_loss_cls"] + o["DA_cst_loss"] + o["tgt_DA_cst_loss"]))


def synthetic_batch(H, W, seed=1, G=8):
    rng = np.random.default_rng(seed)
    means = np.array([102.9801, 115.9465, 122.7717], np.float32)

    def img():
        u8 = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        return torch.from_numpy((u8.astype(np.float32) - means).transpose(2, 0, 1).copy())[None]
    gt = np.zeros((1, 50, 5), np.float32)
    x1, y1 = rng.uniform(0, W - 64, G), rng.uniform(0, H - 64, G)
    w, h = rng.uniform(32, 400, G), rng.uniform(32, 400, G)
    gt[0, :G, 0], gt[0, :G, 1] = x1, y1
    gt[0, :G, 2], gt[0, :G, 3] = np.minimum(x1 + w, W - 1), np.minimum(y1 + h, H - 1)
    gt[0, :G, 4] = rng.integers(1, 9, G)
    info = torch.tensor([[H, W, 600.0 / 1024.0]])
    return (img(), info, torch.from_numpy(gt), torch.tensor([G]), torch.ones(1),
            img(), info.clone(), torch.ones(1, 5), torch.zeros(1, dtype=torch.long), torch.zeros(1))


def time_cpu_steps(steps, H=600, W=1200, warmup=0):
    """Seconds per full DAF step (fwd + bwd + clip + SGD) on the CPU: the median of
    ``steps`` timed steps after ``warmup`` untimed ones (2 + 5)."""
    torch.manual_seed(0)
    m = OracleDAF().train()
    params = [p for p in m.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, lr=2e-3, momentum=0.9, weight_decay=5e-4)
    batch = synthetic_batch(H, W)
    rng = np.random.RandomState(3)
    times = []
    for i in range(warmup + steps):
        t0 = time.perf_counter()
        opt.zero_grad()
        loss = total_loss(m(batch, rng))
        loss.backward()
        tot = torch.sqrt(sum((p.grad.norm() ** 2 for p in params if p.grad is not None)))
        scale = 10.0 / max(float(tot), 10.0)
        for p in params:
            if p.grad is not None:
                p.grad.mul_(scale)
        opt.step()
        if i >= warmup:
            times.append(time.perf_counter() - t0)
    return float(np.median(times))
