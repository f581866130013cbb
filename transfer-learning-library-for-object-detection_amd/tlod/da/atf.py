"""ATF (lib/ATF/{faster_rcnn,vgg16,rpn}.py) on the tlod kernels.

``vgg16(classes).create_architecture()`` then ``model(im_data, im_info, gt_boxes,
num_boxes, need_backprop, tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes,
tgt_need_backprop)`` returns the reference's 12-tuple (lib/ATF/faster_rcnn.py:362-363;
note the order: DA_img, tgt_DA_img, DA_ins, tgt_DA_ins).

ATF keeps two copies of conv3_1..conv5_3: ``RCNN_base`` (the "s" branch) and
``RCNN_base_t`` (deep copies of layers 10+, sharing the frozen conv1/conv2, vgg16.py:
44-64).  Per step the source image runs through both branches, each with its own RPN
losses (the same RCNN_rpn, train mode) and proposal-target sampling; the detection losses
sum over the branches; the source-domain discriminators see the t branch (conv3/4/5 and
the 2000 t-branch proposals through fc6/fc7); the target image runs the s branch with the
RPN in eval mode and TEST post-NMS top-N set to the train count (:259-260).

Scheduling (same math as the reference, fewer passes): conv1/conv2 run once for both
images (frozen, shared); the s branch runs source+target batched; the three RPN heads
(s/src, t/src, s/tgt) run as one batch; the four RoI sets (s sampled, t sampled, t
proposals, target proposals) go through one RoIAlign and one fc6/fc7 pass.  The
reference's unused work — RoIAlign of the s-branch proposals (:185-199) and the target
cls_score (:295-296) — is skipped; it does not feed any output.
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import cfg
from ..rpn.proposal import proposals_on_side_streams
from ..detector.losses import smooth_l1_loss, weighted_loss_sum
from ..rpn.rpn_head import _RPN
from .daf import _ImageDA, _InstanceDA, _fasterRCNN as _DAFBase, image_label
from .daf import early_rpn, early_rpn_backward
from .daf import resnet as _daf_resnet
from .daf import vgg16 as _daf_vgg16
from ..detector.vgg16 import VGG16_SPLITS


def instance_label_f(n_rows, need_backprop, minibatch=256):
    """ATF InstanceLabelResizeLayer (lib/ATF/LabelResizeLayer.py:50-60): float zeros, then
    rows [i*256, (i+1)*256) := need_backprop[i]."""
    nb = need_backprop.view(-1).float()
    y = torch.zeros((n_rows, 1), dtype=torch.float32, device=nb.device)
    for i in range(nb.numel()):
        y[i * minibatch:(i + 1) * minibatch] = nb[i]
    return y


class _fasterRCNN(_DAFBase):
    """lib/ATF/faster_rcnn.py:84-389."""

    def __init__(self, classes, class_agnostic):
        super().__init__(classes, class_agnostic)
        del self.consistency_loss
        # RCNN_rpn_t is built by the reference (:95) but never called: it keeps its init
        # weights (SGD skips parameters without gradients) — frozen here to the same effect
        self.RCNN_rpn_t = _RPN(self.dout_base_model)
        for p in self.RCNN_rpn_t.parameters():
            p.requires_grad = False
        self.RCNN_imageDA_3 = _ImageDA(256)  # VGG conv3_3 / ResNet layer1: 256 channels
        self.RCNN_imageDA_4 = _ImageDA(512)  # VGG conv4_3 / ResNet layer2: 512 channels
        self.RCNN_imageDA = _ImageDA(self.dout_base_model)
        self.RCNN_instanceDA = _InstanceDA(self.instance_dim)

    def _shared(self, x):
        """The frozen prefix both branches share (VGG16 conv1/conv2; ResNet conv1..layer1)."""
        return self.RCNN_base[:self.splits[0]](x)

    def _branch(self, layers, z):
        shared, e3, e4 = self.splits
        c3 = layers[shared:e3](z) if e3 > shared else z
        c4 = layers[e3:e4](c3)
        return c3, c4, layers[e4:](c4)

    @staticmethod
    def _img_loss(score, need):
        return F.nll_loss(F.log_softmax(score, 1), image_label(score, need), ignore_index=-1)

    def _sampled(self, rois, gt_boxes, num_boxes):
        rois, label, target, inside, outside = self.RCNN_proposal_target(
            rois, gt_boxes, num_boxes, rng=self.replay_rng)
        return (rois, label.view(-1).long(), target.view(-1, target.size(2)),
                inside.view(-1, inside.size(2)), outside.view(-1, outside.size(2)))

    def forward(self, im_data, im_info, gt_boxes, num_boxes, need_backprop,
                tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes, tgt_need_backprop):
        batch_size = im_data.size(0)
        im_info = im_info.detach()
        gt_boxes = gt_boxes.detach()
        same = (im_data.shape == tgt_im_data.shape) and batch_size == 1
        rpn = self.RCNN_rpn
        early = early_rpn(self, same)

        # ---- backbones: frozen conv1/conv2 are shared by both branches (vgg16.py:46-47)
        if same:
            z = self._shared(torch.cat([im_data, tgt_im_data], 0))
            c3s, c4s, bs = self._branch(self.RCNN_base, z)
            c3_t, c4_t, base_t = self._branch(self.RCNN_base_t, z[:1])
            base_feat, tgt_base_feat = bs[:1], bs[1:]
            tgt_c3, tgt_c4 = c3s[1:], c4s[1:]
            rpn_in = torch.cat([base_feat, base_t, tgt_base_feat], 0)
            if early:
                rpn_in = rpn_in.detach().requires_grad_(True)
            heads = rpn.head(rpn_in)
            hs = [tuple(h[i:i + 1] for h in heads) for i in range(3)]
        else:
            z = self._shared(im_data)
            _, _, base_feat = self._branch(self.RCNN_base, z)
            c3_t, c4_t, base_t = self._branch(self.RCNN_base_t, z)
            tgt_c3, tgt_c4, tgt_base_feat = self._branch(self.RCNN_base, self._shared(tgt_im_data))
            hs = [rpn.head(f) for f in (base_feat, base_t, tgt_base_feat)]

        # ---- RPN, train mode, on the source image through both branches (:130-134)
        # target image: eval-mode RPN with TEST post-NMS top-N := the train count (:258-260,
        # rois_domain.size(1)); the three proposal layers run on side streams while this
        # stream computes the two RPN losses
        cfg.TEST.RPN_POST_NMS_TOP_N = cfg.TRAIN.RPN_POST_NMS_TOP_N
        pending = proposals_on_side_streams(rpn.RPN_proposal, [
            (hs[0][2].detach(), hs[0][3].detach(), im_info, "TRAIN"),
            (hs[1][2].detach(), hs[1][3].detach(), im_info, "TRAIN"),
            (hs[2][2].detach(), hs[2][3].detach(), tgt_im_info.detach(), "TEST")])
        l_cls1, l_box1, _ = rpn.losses(hs[0][0], hs[0][1], hs[0][3], gt_boxes, im_info, num_boxes,
                                       rng=self.replay_rng)
        l_cls2, l_box2, _ = rpn.losses(hs[1][0], hs[1][1], hs[1][3], gt_boxes, im_info, num_boxes,
                                       rng=self.replay_rng)
        rpn_loss_cls = l_cls1 + l_cls2
        rpn_loss_bbox = l_box1 + l_box2
        if early:  # rpn_in rows: source (RCNN_base), source (RCNN_base_t), target (RCNN_base)
            rpn_loss_cls, rpn_loss_bbox = early_rpn_backward(
                rpn_loss_cls, rpn_loss_bbox, rpn_in,
                [(bs, lambda g: torch.cat([g[0:1], g[2:3]], 0)), (base_t, lambda g: g[1:2])])
        rois_domain, rois_domain_t, tgt_rois = pending.join()
        if self.capture is not None:
            self.capture.update(s_rois=rois_domain.detach().clone(),
                                st_rois=rois_domain_t.detach().clone(),
                                t_rois=tgt_rois.detach().clone())

        rois, rois_label, rois_target, rois_inside_ws, rois_outside_ws = \
            self._sampled(rois_domain, gt_boxes, num_boxes)
        rois_t, rois_label_t, rois_target_t, rois_inside_ws_t, rois_outside_ws_t = \
            self._sampled(rois_domain_t, gt_boxes, num_boxes)

        # ---- one RoIAlign + fc6/fc7 pass over the four RoI sets
        sets = (rois, rois_t, rois_domain_t, tgt_rois)
        n = [r.size(1) for r in sets]
        if same:
            feats = torch.cat([base_feat, tgt_base_feat, base_t], 0)
            idx = (0, 2, 2, 1)
            rr = []
            for r, i in zip(sets, idx):
                r = r.view(-1, 5).clone()
                r[:, 0] = float(i)
                rr.append(r)
            fc7 = self._head_to_tail(self._pool(feats, torch.cat(rr, 0)))
        else:
            maps = (base_feat, base_t, base_t, tgt_base_feat)
            fc7 = torch.cat([self._head_to_tail(self._pool(f, r.view(-1, 5)))
                             for f, r in zip(maps, sets)], 0)
        o = [0]
        for k in n:
            o.append(o[-1] + k)
        det = fc7[:o[2]]  # s-branch and t-branch sampled RoIs

        bbox_all = self.RCNN_bbox_pred(det)
        labels = torch.cat([rois_label, rois_label_t])
        if self.training and not self.class_agnostic:
            view = bbox_all.view(bbox_all.size(0), int(bbox_all.size(1) / 4), 4)
            bbox_all = torch.gather(view, 1, labels.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        cls_all = self.RCNN_cls_score(det)
        RCNN_loss_cls = (F.cross_entropy(cls_all[:n[0]], rois_label)
                         + F.cross_entropy(cls_all[n[0]:], rois_label_t))
        RCNN_loss_bbox = (smooth_l1_loss(bbox_all[:n[0]], rois_target, rois_inside_ws,
                                         rois_outside_ws)
                          + smooth_l1_loss(bbox_all[n[0]:], rois_target_t, rois_inside_ws_t,
                                           rois_outside_ws_t))
        cls_prob = F.softmax(cls_all[:n[0]], 1).view(batch_size, rois_t.size(1), -1)
        bbox_pred = bbox_all[:n[0]].view(batch_size, rois_t.size(1), -1)

        # ---- image DA: source through the t branch, target through the s branch (:306-354)
        da_heads = (self.RCNN_imageDA_3, self.RCNN_imageDA_4, self.RCNN_imageDA)
        if same:
            pairs = ((c3_t, tgt_c3), (c4_t, tgt_c4), (base_t, tgt_base_feat))
            sc = [h(torch.cat(p, 0), need_backprop.new_ones(2))[0] for h, p in zip(da_heads, pairs)]
            s_scores, t_scores = [s[:1] for s in sc], [s[1:] for s in sc]
        else:
            s_scores = [h(f, need_backprop)[0] for h, f in zip(da_heads, (c3_t, c4_t, base_t))]
            t_scores = [h(f, tgt_need_backprop)[0]
                        for h, f in zip(da_heads, (tgt_c3, tgt_c4, tgt_base_feat))]
        DA_img_loss_cls = sum(self._img_loss(s, need_backprop) for s in s_scores)
        tgt_DA_img_loss_cls = sum(self._img_loss(s, tgt_need_backprop) for s in t_scores)

        # ---- instance DA: t-branch proposals (source) and target proposals (:326-345)
        ins, _ = self.RCNN_instanceDA(fc7[o[2]:], need_backprop.new_ones(1))
        ins_s, ins_t = ins[:n[2]], ins[n[2]:]
        DA_ins_loss_cls = F.binary_cross_entropy(ins_s, instance_label_f(n[2], need_backprop))
        tgt_DA_ins_loss_cls = F.binary_cross_entropy(ins_t, instance_label_f(n[3], tgt_need_backprop))
        return (rois_t, cls_prob, bbox_pred, rpn_loss_cls, rpn_loss_bbox, RCNN_loss_cls,
                RCNN_loss_bbox, rois_label_t, DA_img_loss_cls, tgt_DA_img_loss_cls,
                DA_ins_loss_cls, tgt_DA_ins_loss_cls)

    @staticmethod
    def total_loss(out, lamda=0.1):
        """methods/ATF/ATF_train.py:405-408 (image DA weighted 7x)."""
        (_, _, _, rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, _, DA_img,
         tgt_DA_img, DA_ins, tgt_DA_ins) = out
        return weighted_loss_sum(
            (rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, DA_img, DA_ins, tgt_DA_img,
             tgt_DA_ins), (1, 1, 1, 1, lamda * 7, lamda, lamda * 7, lamda))


class vgg16(_fasterRCNN):
    """lib/ATF/vgg16.py:20-79."""

    FUSE_POOLS = (1, 2)  # the DA taps read conv3 / conv4 before pools 3 / 4

    def __init__(self, classes, pretrained=False, class_agnostic=False):
        self.dout_base_model = 512
        self.instance_dim = 4096
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    splits = VGG16_SPLITS

    def _init_modules(self):
        _daf_vgg16._init_modules(self)
        _make_t_branch(self)

    def _head_to_tail(self, pool5):
        return self.RCNN_top(pool5.view(pool5.size(0), -1))


def _make_t_branch(m):
    """RCNN_base_t: the frozen prefix shared, the rest deep-copied (vgg16.py:44-50), and
    the conv3/conv34/conv45 _s/_t views (:52-59)."""
    shared, e3, e4 = m.splits
    layers = list(m.RCNN_base)
    m.RCNN_base_t = type(m.RCNN_base)(*(layers[:shared] + [copy.deepcopy(x) for x in layers[shared:]]))
    for tag, base in (("s", m.RCNN_base), ("t", m.RCNN_base_t)):
        setattr(m, "conv3_" + tag, base[:e3])
        setattr(m, "conv34_" + tag, base[e3:e4])
        setattr(m, "conv45_" + tag, base[e4:])


class resnet(_fasterRCNN):
    """ATF with ResNet101.  The reference's lib/ATF/resnet.py cannot run (its forward needs
    conv3_s/_t... which only ATF/vgg16.py defines): built here the way the
    VGG16 variant is, with the taps conv1..layer1 | layer2 | layer3 (ATF/resnet.py:238-241),
    the frozen conv1..layer1 shared and layer2/layer3 copied for the t branch, and the
    instance head on the 2048-d features.  Parity is against the oracle restatement only."""

    splits = None

    def __init__(self, classes, num_layers=101, pretrained=False, class_agnostic=False):
        if num_layers != 101:
            raise NotImplementedError("only ResNet101")
        self.dout_base_model = 1024
        self.instance_dim = 2048
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    def _init_modules(self):
        _daf_resnet._init_modules(self)
        self.splits = self.RCNN_base.SPLITS
        _make_t_branch(self)

    train = _daf_resnet.train
    _head_to_tail = _daf_resnet._head_to_tail
    _pool = _daf_resnet._pool
