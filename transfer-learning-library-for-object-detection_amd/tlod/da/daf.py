"""DAF (Domain Adaptive Faster R-CNN) on the tlod kernels — lib/DAF/{DA,faster_rcnn,vgg16}.py.

``vgg16(classes).create_architecture()`` then ``model(im_data, im_info, gt_boxes,
num_boxes, need_backprop, tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes,
tgt_need_backprop)`` returns the reference's 14-tuple (lib/DAF/faster_rcnn.py:222-223).

Execution differs from the reference only in scheduling, not in math:
  * source and target images share one backbone / RPN-conv / RoIAlign / head pass
    (batched along N) when their sizes match — every op is per-image, so the results
    are the same as two passes (the reference runs RCNN_base twice, :58 and :137);
  * the DA label layers (LabelResizeLayer.py:18-57: D2H, cv2.resize, H2D) become
    on-device constant fills, including the reference's instance-label quirk (target
    RoIs 256.. get label 1 because only the first 256 rows are overwritten, :48-55);
  * no host synchronisation anywhere in the step (nonzero / .item() / numpy RNG are
    replaced by device-side equivalents, see tlod.rpn).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..config import cfg
from ..conv import Conv2d
from ..linear import Linear, relu_dropout
from ..detector.losses import (daf_da_losses, daf_da_losses_packed, fused_losses, rcnn_losses,
                               smooth_l1_loss, weighted_loss_sum)
from ..detector.vgg16 import vgg16_base, vgg16_top
from ..roi_align import RoIAlignAvg
from ..roi_pool import _RoIPooling
from ..rpn.proposal import proposals_on_side_streams
from ..rpn.proposal_target import _ProposalTargetLayer
from ..rpn.rpn_head import _RPN


class GRLayer(torch.autograd.Function):
    """Gradient reversal (lib/DAF/DA.py:19-33): identity forward, -alpha * grad backward."""

    @staticmethod
    def forward(ctx, x, alpha=0.1):
        ctx.alpha = alpha
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * (-ctx.alpha), None  # = g.neg() * alpha bit for bit (negation is exact)


def grad_reverse(x, alpha=0.1):
    return GRLayer.apply(x, alpha)


def image_label(score, need_backprop):
    """ImageLabelResizeLayer (LabelResizeLayer.py:18-38): (B,H,W) long filled with the
    per-image need_backprop — on device."""
    B, _, H, W = score.shape
    return need_backprop.view(-1, 1, 1).to(score.device).long().expand(B, H, W)


def instance_label(n_rows, need_backprop, minibatch=256):
    """InstanceLabelResizeLayer (LabelResizeLayer.py:41-57): ones, then rows
    [i*256, (i+1)*256) := need_backprop[i] (rows past B*256 stay 1)."""
    nb = need_backprop.view(-1).float()
    y = torch.ones((n_rows, 1), dtype=torch.float32, device=nb.device)
    for i in range(nb.numel()):
        y[i * minibatch:(i + 1) * minibatch] = nb[i]
    return y


class _ImageDA(nn.Module):
    """lib/DAF/DA.py:36-50: GRL -> 1x1 dim->512 -> ReLU -> 1x1 512->2 (no biases)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.Conv1 = Conv2d(dim, 512, 1, bias=False, relu=True)
        self.Conv2 = Conv2d(512, 2, 1, bias=False)

    def score(self, x):
        """The domain logits alone (the DAF forward discards the label tensor)."""
        return self.Conv2(self.Conv1(grad_reverse(x)))

    def forward(self, x, need_backprop):
        x = self.score(x)
        return x, image_label(x, need_backprop)


class _InstanceDA(nn.Module):
    """lib/DAF/DA.py:53-73: GRL -> fc 1024 -> fc 1024 -> fc 1 -> sigmoid.

    ``in_dim`` is 4096 for VGG16 (the reference hard-codes 4096, which breaks its
    ResNet101 variant whose head emits 2048-d features, lib/DAF/resnet.py:243)."""

    def __init__(self, in_dim=4096):
        super().__init__()
        self.dc_ip1 = Linear(in_dim, 1024)
        self.dc_relu1 = nn.ReLU()
        self.dc_drop1 = nn.Dropout(p=0.5)
        self.dc_ip2 = Linear(1024, 1024)
        self.dc_relu2 = nn.ReLU()
        self.dc_drop2 = nn.Dropout(p=0.5)
        self.clssifer = nn.Linear(1024, 1)

    def score(self, x):
        """The sigmoid outputs alone (the DAF forward discards the label tensor)."""
        x = grad_reverse(x)
        x = relu_dropout(self.dc_ip1(x), self.dc_drop1, getattr(self.dc_ip1, "act_tap", None))
        x = relu_dropout(self.dc_ip2(x), self.dc_drop2, getattr(self.dc_ip2, "act_tap", None))
        return torch.sigmoid(self.clssifer(x))

    def forward(self, x, need_backprop):
        x = self.score(x)
        return x, instance_label(x.shape[0], need_backprop)


def early_rpn(model, same):
    """Early RPN backward (round 6): the RPN losses do not depend on the proposals, so their
    backward (RPN head + RPN_Conv weight / input gradients) can run on the main stream while
    the proposal layers' NMS runs on the side streams — the window in which the main stream
    otherwise waits at pending.join() with the chip nearly idle.  The RPN head then reads a
    detached copy of its input, and early_rpn_backward adds the input gradient to the
    features' gradients by hooks in the main backward.  The returned RPN losses are detached:
    their gradient, at weight 1 as in the reference's loss sums (methods/DAF/DAF_train.py:
    397-400, MAF_train.py:415-418, ATF_train.py:405-408), is already in the RPN parameters'
    .grad, so a caller that weights them differently or runs a training forward without its
    backward sets TLOD_EARLY_RPN=0 (one backward).  Only on the batched (same-shape, batch 1)
    path."""
    return (same and model.training and torch.is_grad_enabled()
            and _lib.env("TLOD_EARLY_RPN", "1") != "0")


def early_rpn_backward(loss_cls, loss_bbox, rpn_in, targets):
    """Backpropagates the RPN losses now.  rpn_in: the detached leaf the RPN head read;
    targets: (feature, share) pairs — share(rpn_in.grad) is the part of that gradient which
    belongs to the feature (a slice / concatenation of rows), added to the feature's gradient
    when the main backward reaches it.  Returns the detached losses."""
    torch.autograd.backward(loss_cls + loss_bbox)
    g = rpn_in.grad
    if g is not None:
        for feat, share in targets:
            if feat.requires_grad:
                gs = share(g)
                feat.register_hook(lambda gf, gs=gs: gf + gs)
    return loss_cls.detach(), loss_bbox.detach()


class _fasterRCNN(nn.Module):
    """lib/DAF/faster_rcnn.py:22-247."""

    def __init__(self, classes, class_agnostic):
        super().__init__()
        self.classes = classes
        self.n_classes = len(classes)
        self.class_agnostic = class_agnostic
        self.RCNN_loss_cls = 0
        self.RCNN_loss_bbox = 0
        self.RCNN_rpn = _RPN(self.dout_base_model)
        self.RCNN_proposal_target = _ProposalTargetLayer(self.n_classes)
        self.RCNN_roi_pool = _RoIPooling(cfg.POOLING_SIZE, cfg.POOLING_SIZE, 1.0 / 16.0)
        self.RCNN_roi_align = RoIAlignAvg(cfg.POOLING_SIZE, cfg.POOLING_SIZE, 1.0 / 16.0)
        self.RCNN_imageDA = _ImageDA(self.dout_base_model)
        self.RCNN_instanceDA = _InstanceDA(self.instance_dim)
        self.consistency_loss = nn.MSELoss(reduction="sum")
        self.replay_rng = None  # tests: np.random-like object -> reference-exact sampling
        self.capture = None     # tests: dict receiving the proposal-layer rois

    # ------------------------------------------------------------------ pieces
    def _pool(self, feat, rois):
        if cfg.POOLING_MODE == "align":
            return self.RCNN_roi_align(feat, rois)
        if cfg.POOLING_MODE == "pool":
            return self.RCNN_roi_pool(feat, rois)
        raise NotImplementedError("POOLING_MODE 'crop' is out of scope (configs use 'align')")

    def _rcnn_losses(self, pooled_s, rois_label, rois_target, rois_inside_ws, rois_outside_ws):
        """Head outputs and losses of the first rois_label.numel() rows of ``pooled_s``
        (the source RoIs; the batched pass appends the target RoIs, whose head outputs
        are unused)."""
        bbox_pred = self.RCNN_bbox_pred(pooled_s)
        if self.training and fused_losses():
            return rcnn_losses(self.RCNN_cls_score(pooled_s), bbox_pred, rois_label, rois_target,
                               rois_inside_ws, rois_outside_ws, self.class_agnostic)
        n_s = rois_label.numel()
        pooled_s, bbox_pred = pooled_s[:n_s], bbox_pred[:n_s]
        if self.training and not self.class_agnostic:
            view = bbox_pred.view(bbox_pred.size(0), int(bbox_pred.size(1) / 4), 4)
            bbox_pred = torch.gather(view, 1, rois_label.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        cls_score = self.RCNN_cls_score(pooled_s)
        cls_prob = F.softmax(cls_score, 1)
        loss_cls = F.cross_entropy(cls_score, rois_label)
        loss_bbox = smooth_l1_loss(bbox_pred, rois_target, rois_inside_ws, rois_outside_ws)
        return cls_prob, bbox_pred, loss_cls, loss_bbox

    def _da_losses(self, base_score_s, base_score_t, ins_s, ins_t, need_s, need_t):
        if fused_losses():
            return daf_da_losses(base_score_s, base_score_t, ins_s, ins_t, need_s, need_t)
        lab_s = image_label(base_score_s, need_s)
        lab_t = image_label(base_score_t, need_t)
        da_img = F.nll_loss(F.log_softmax(base_score_s, 1), lab_s)
        tgt_da_img = F.nll_loss(F.log_softmax(base_score_t, 1), lab_t)
        y_s = instance_label(ins_s.shape[0], need_s)
        y_t = instance_label(ins_t.shape[0], need_t)
        da_ins = F.binary_cross_entropy(ins_s, y_s)
        tgt_da_ins = F.binary_cross_entropy(ins_t, y_t)
        cons_s = F.softmax(base_score_s, 1)[:, 1, :, :].mean()
        cons_t = F.softmax(base_score_t, 1)[:, 0, :, :].mean()
        da_cst = self.consistency_loss(ins_s, cons_s.detach().expand_as(ins_s))
        tgt_da_cst = self.consistency_loss(ins_t, cons_t.detach().expand_as(ins_t))
        return da_img, da_ins, tgt_da_img, tgt_da_ins, da_cst, tgt_da_cst

    # ------------------------------------------------------------------ forward
    def forward(self, im_data, im_info, gt_boxes, num_boxes, need_backprop,
                tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes, tgt_need_backprop):
        batch_size = im_data.size(0)
        im_info = im_info.detach()
        gt_boxes = gt_boxes.detach()
        same = (im_data.shape == tgt_im_data.shape) and batch_size == 1
        early = early_rpn(self, same)
        if same:
            base2 = self.RCNN_base(torch.cat([im_data, tgt_im_data], 0))
            base_feat, tgt_base_feat = base2[:1], base2[1:]
            rpn_in = base2.detach().requires_grad_(True) if early else base2
            score2, score_r2, prob2, bbox2 = self.RCNN_rpn.head(rpn_in)
            s_score, s_score_r, s_prob, s_bbox = score2[:1], score_r2[:1], prob2[:1], bbox2[:1]
            t_prob, t_bbox = prob2[1:], bbox2[1:]
        else:
            base_feat = self.RCNN_base(im_data)
            tgt_base_feat = self.RCNN_base(tgt_im_data)
            s_score, s_score_r, s_prob, s_bbox = self.RCNN_rpn.head(base_feat)
            _, _, t_prob, t_bbox = self.RCNN_rpn.head(tgt_base_feat)

        # source RPN in train mode (faster_rcnn.py:62-63); target RPN in eval mode
        # (faster_rcnn.py:140-142): TEST proposals, no losses.  The two proposal layers run
        # on side streams while this stream does the anchor target, RPN losses and the
        # image-level DA head (independent of the proposals).
        rpn = self.RCNN_rpn
        pending = proposals_on_side_streams(rpn.RPN_proposal, [
            (s_prob.detach(), s_bbox.detach(), im_info, "TRAIN"),
            (t_prob.detach(), t_bbox.detach(), tgt_im_info.detach(), "TEST")])
        if same:  # the source image's losses over the batched head outputs
            rpn_loss_cls, rpn_loss_bbox, _ = rpn.losses(score2, score_r2, bbox2, gt_boxes, im_info,
                                                        num_boxes, rng=self.replay_rng, n_images=1)
        else:
            rpn_loss_cls, rpn_loss_bbox, _ = rpn.losses(s_score, s_score_r, s_bbox, gt_boxes,
                                                        im_info, num_boxes, rng=self.replay_rng)
        if early:
            rpn_loss_cls, rpn_loss_bbox = early_rpn_backward(
                rpn_loss_cls, rpn_loss_bbox, rpn_in, [(base2, lambda g: g)])
        if same:
            score_img2 = self.RCNN_imageDA.score(base2)
        rois, tgt_rois = pending.join()
        if self.capture is not None:
            self.capture.update(s_rois=rois.detach().clone(), t_rois=tgt_rois.detach().clone())

        rois, rois_label, rois_target, rois_inside_ws, rois_outside_ws = \
            self.RCNN_proposal_target(rois, gt_boxes, num_boxes, rng=self.replay_rng)
        rois_label = rois_label.view(-1).long()
        rois_target = rois_target.view(-1, rois_target.size(2))
        rois_inside_ws = rois_inside_ws.view(-1, rois_inside_ws.size(2))
        rois_outside_ws = rois_outside_ws.view(-1, rois_outside_ws.size(2))

        n_s = rois.size(1)
        if same:
            t_rois = tgt_rois.view(-1, 5).clone()
            t_rois[:, 0] = 1.0  # target image is batch entry 1 of base2
            pooled2 = self._pool(base2, torch.cat([rois.view(-1, 5), t_rois], 0))
            feat2 = self._head_to_tail(pooled2)
            pooled_feat, tgt_pooled_feat = feat2[:n_s], feat2[n_s:]
        else:
            pooled_feat = self._head_to_tail(self._pool(base_feat, rois.view(-1, 5)))
            tgt_pooled_feat = self._head_to_tail(self._pool(tgt_base_feat, tgt_rois.view(-1, 5)))

        cls_prob, bbox_pred, RCNN_loss_cls, RCNN_loss_bbox = self._rcnn_losses(
            feat2 if same else pooled_feat, rois_label, rois_target, rois_inside_ws,
            rois_outside_ws)
        cls_prob = cls_prob.view(batch_size, n_s, -1)
        bbox_pred = bbox_pred.view(batch_size, n_s, -1)

        # DA heads (faster_rcnn.py:181-220)
        if same:
            ins2 = self.RCNN_instanceDA.score(feat2)
            if fused_losses():
                da = daf_da_losses_packed(score_img2, ins2, 1, n_s, need_backprop,
                                          tgt_need_backprop)
            else:
                da = self._da_losses(score_img2[:1], score_img2[1:], ins2[:n_s], ins2[n_s:],
                                     need_backprop, tgt_need_backprop)
        else:
            base_score = self.RCNN_imageDA.score(base_feat)
            tgt_base_score = self.RCNN_imageDA.score(tgt_base_feat)
            ins_s = self.RCNN_instanceDA.score(pooled_feat)
            ins_t = self.RCNN_instanceDA.score(tgt_pooled_feat)
            da = self._da_losses(base_score, tgt_base_score, ins_s, ins_t, need_backprop,
                                 tgt_need_backprop)
        DA_img_loss_cls, DA_ins_loss_cls, tgt_DA_img_loss_cls, tgt_DA_ins_loss_cls, \
            DA_cst_loss, tgt_DA_cst_loss = da
        return (rois, cls_prob, bbox_pred, rpn_loss_cls, rpn_loss_bbox, RCNN_loss_cls,
                RCNN_loss_bbox, rois_label, DA_img_loss_cls, DA_ins_loss_cls, tgt_DA_img_loss_cls,
                tgt_DA_ins_loss_cls, DA_cst_loss, tgt_DA_cst_loss)

    @staticmethod
    def total_loss(out, lamda=0.1):
        """methods/DAF/DAF_train.py:397-400."""
        (_, _, _, rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, _, DA_img, DA_ins,
         tgt_DA_img, tgt_DA_ins, DA_cst, tgt_DA_cst) = out
        return weighted_loss_sum(
            (rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, DA_img, DA_ins, tgt_DA_img,
             tgt_DA_ins, DA_cst, tgt_DA_cst), (1, 1, 1, 1) + (lamda,) * 6)

    def _init_weights(self):
        """faster_rcnn.py:227-243 (normal_init, truncated=False)."""
        def normal_init(m, mean, std):
            m.weight.data.normal_(mean, std)
            m.bias.data.zero_()
        normal_init(self.RCNN_rpn.RPN_Conv, 0, 0.01)
        normal_init(self.RCNN_rpn.RPN_cls_score, 0, 0.01)
        normal_init(self.RCNN_rpn.RPN_bbox_pred, 0, 0.01)
        normal_init(self.RCNN_cls_score, 0, 0.01)
        normal_init(self.RCNN_bbox_pred, 0, 0.001)

    def create_architecture(self):
        self._init_modules()
        self._init_weights()


class vgg16(_fasterRCNN):
    """lib/DAF/vgg16.py:20-71 (random init: pretrained caffe weights are external)."""

    def __init__(self, classes, pretrained=False, class_agnostic=False):
        self.dout_base_model = 512
        self.instance_dim = 4096
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    # max-pools folded into the preceding conv (tlod.detector.vgg16.vgg16_base); MAF / ATF,
    # whose DA taps read the conv3 / conv4 outputs, keep pools 3 and 4 separate
    FUSE_POOLS = (1, 2, 3, 4)

    def _init_modules(self):
        self.RCNN_base = vgg16_base(fuse_pools=self.FUSE_POOLS)
        self.RCNN_top = vgg16_top()
        self.RCNN_cls_score = nn.Linear(4096, self.n_classes)
        self.RCNN_bbox_pred = nn.Linear(4096, 4 if self.class_agnostic else 4 * self.n_classes)

    def _head_to_tail(self, pool5):
        return self.RCNN_top(pool5.view(pool5.size(0), -1))


class resnet(_fasterRCNN):
    """lib/DAF/resnet.py:220-288 (ResNet101; random init — the caffe weights are external).

    Deviation, documented: the reference's _InstanceDA is Linear(4096, ...) (DA.py:56)
    and crashes on the 2048-d ResNet head features; here the instance head takes 2048."""

    def __init__(self, classes, num_layers=101, pretrained=False, class_agnostic=False):
        if num_layers != 101:
            raise NotImplementedError("only ResNet101 (the reference's only depth)")
        self.dout_base_model = 1024
        self.instance_dim = 2048
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    def _init_modules(self):
        from ..detector.resnet import resnet101_parts
        self.RCNN_base, self.RCNN_top = resnet101_parts(cfg.RESNET.FIXED_BLOCKS)
        self.RCNN_cls_score = nn.Linear(2048, self.n_classes)
        self.RCNN_bbox_pred = nn.Linear(2048, 4 if self.class_agnostic else 4 * self.n_classes)

    def train(self, mode=True):
        """resnet.py:269-284: BatchNorm stays in eval mode."""
        nn.Module.train(self, mode)
        if mode:
            from ..detector.resnet import set_bn_eval
            set_bn_eval(self.RCNN_base)
            set_bn_eval(self.RCNN_top)
        return self

    def _pool(self, feat, rois):
        # pool5 feeds only RCNN_top: the head entry (bins (2i, 2j), channels-last)
        from ..detector.resnet import resnet_pool
        return resnet_pool(self, feat, rois, _fasterRCNN._pool)

    def _head_to_tail(self, pool5):
        # RCNN_top(pool5).mean(3).mean(2) (resnet.py:286-288); the head runs channels-last
        return self.RCNN_top(pool5, mean=True)
