"""MAF (multi-adversarial Faster R-CNN) on the tlod kernels — lib/MAF/{drm,DA,
faster_rcnn,vgg16}.py.

``vgg16(classes).create_architecture()`` then ``model(im_data, im_info, gt_boxes,
num_boxes, need_backprop, tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes,
tgt_need_backprop)`` returns the reference's 12-tuple (lib/MAF/faster_rcnn.py:247-248).

Beyond DAF: image discriminators on conv3 and conv4 through the DRM (1x1 conv + ReLU +
crop + space-to-depth, drm.py:10-42), and a weighted-GRL instance discriminator on
[fc7 || cls_prob] (4105-d for VGG16, DA.py:78-104).  As in tlod.da.daf, source and
target share each batched pass when their sizes match (per-image ops: same math), the
label layers are device fills, and the WGRL weights (DA.py:45-53: a .cpu() of the domain
label per backward) are a per-row device tensor.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..conv import Conv2d
from ..detector.losses import weighted_loss_sum
from ..linear import Linear
from ..rpn.proposal import proposals_on_side_streams
from .daf import _ImageDA, _fasterRCNN as _DAFBase, grad_reverse, image_label
from .daf import early_rpn, early_rpn_backward
from .daf import resnet as _daf_resnet
from .daf import vgg16 as _daf_vgg16
from ..detector.vgg16 import VGG16_SPLITS


class SpaceToDepthFunction(torch.autograd.Function):
    """DRM's chunk/reshape/cat (drm.py:23-40) as one libtlod permutation each way."""

    @staticmethod
    def forward(ctx, x, scale):
        _lib.require_cuda(x)
        x = x.contiguous()
        B, C, H, W = x.shape
        s = int(scale)
        y = torch.empty((B, C * s * s, H // s, W // s), dtype=x.dtype, device=x.device)
        _lib.check(_lib.lib().tlod_space_to_depth_f32(_lib.ptr(x), B, C, H, W, s, _lib.ptr(y),
                                                      _lib.stream_of(x)), "space_to_depth")
        ctx.meta = (B, C, H, W, s)
        return y

    @staticmethod
    def backward(ctx, g):
        B, C, H, W, s = ctx.meta
        g = g.contiguous()
        dx = torch.empty((B, C, H, W), dtype=g.dtype, device=g.device)
        _lib.check(_lib.lib().tlod_depth_to_space_f32(_lib.ptr(g), B, C, H, W, s, _lib.ptr(dx),
                                                      _lib.stream_of(g)), "depth_to_space")
        return dx, None


def space_to_depth(x, scale):
    return SpaceToDepthFunction.apply(x, scale)


class DRMFunction(torch.autograd.Function):
    """The whole DRM (drm.py:10-42: conv_low_dim 1x1 without bias -> ReLU -> crop ->
    space-to-depth) as one conv launch whose epilogue stores every output at its
    space-to-depth position (tlod_drm_fwd_f32; the (B, C, H, W) map is never written), and
    its backward as one depth-to-space + ReLU-mask pass (tlod_drm_relu_bwd_f32) ahead of the
    1x1 dgrad / wgrad."""

    @staticmethod
    def forward(ctx, x, weight, scale, tap=None):
        from ..conv import _check, pack_fwd
        _check(x, weight)
        x = x.contiguous()
        B, Cin, H, W = x.shape
        C, s = weight.shape[0], int(scale)
        L = _lib.lib()
        y = torch.empty((B, C * s * s, H // s, W // s), dtype=x.dtype, device=x.device)
        ws = _lib.workspace(L.tlod_conv_fwd_workspace_bytes(B, Cin, H, W, C, 1), x.device, "conv")
        _lib.check(L.tlod_drm_fwd_f32(_lib.ptr(x), _lib.ptr(pack_fwd(weight)), _lib.ptr(y), B, Cin,
                                      H, W, C, s, _lib.ptr(ws), ws.numel(), _lib.stream_of(x)),
                   "drm_fwd")
        if tap is not None:  # test instrumentation: the ReLU map (0 on the cropped border)
            m = torch.empty((B, C, H, W), dtype=y.dtype, device=y.device)
            _lib.check(L.tlod_depth_to_space_f32(_lib.ptr(y), B, C, H, W, s, _lib.ptr(m),
                                                 _lib.stream_of(y)), "depth_to_space")
            tap.append(m)
        ctx.meta = (B, C, H, W, s)
        ctx.wparam = weight
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..conv import conv_dgrad, conv_wgrad
        from ..grads import grad_out
        x, weight, y = ctx.saved_tensors
        B, C, H, W, s = ctx.meta
        dy = dy.contiguous()
        g = torch.empty((B, C, H, W), dtype=dy.dtype, device=dy.device)
        _lib.check(_lib.lib().tlod_drm_relu_bwd_f32(_lib.ptr(dy), _lib.ptr(y), B, C, H, W, s,
                                                    _lib.ptr(g), _lib.stream_of(dy)),
                   "drm_relu_bwd")
        dx = conv_dgrad(g, weight) if ctx.needs_input_grad[0] else None
        dw = conv_wgrad(g, x, 1, out=grad_out(ctx.wparam)) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None


class DRM(nn.Module):
    """lib/MAF/drm.py:10-42; conv_low_dim (1x1, no bias) keeps the reference's module and
    state_dict key, its ReLU, crop and space-to-depth run fused (DRMFunction)."""

    def __init__(self, in_dim, inner_channel, scale):
        super().__init__()
        self.in_dim, self.inner_channel, self.scale = in_dim, inner_channel, scale
        self.conv_low_dim = Conv2d(in_dim, inner_channel, 1, bias=False, relu=True)

    def forward(self, x):
        return DRMFunction.apply(x, self.conv_low_dim.weight, self.scale,
                                 self.conv_low_dim.act_tap)


class WGRLayer(torch.autograd.Function):
    """lib/MAF/DA.py:34-53: identity forward; backward -alpha * w[row] * grad, w[row] =
    the (detached) discriminator probability of the row's own domain."""

    @staticmethod
    def forward(ctx, x, weight, alpha=0.2):
        ctx.save_for_backward(weight)
        ctx.alpha = alpha
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        return g.neg() * w.view(-1, 1) * ctx.alpha, None, None


def wgrad_reverse(x, weight, alpha=0.2):
    return WGRLayer.apply(x, weight, alpha)


def instance_label_w(n_rows, need_backprop, minibatch=256):
    """MAF InstanceLabelResizeLayer (lib/MAF/LabelResizeLayer.py:50-60): zeros, then rows
    [i*256, (i+1)*256) := need_backprop[i]; long."""
    nb = need_backprop.view(-1)
    y = torch.zeros(n_rows, dtype=torch.long, device=nb.device)
    for i in range(nb.numel()):
        y[i * minibatch:(i + 1) * minibatch] = nb[i].long()
    return y


def _row_domain(need_backprop, n_rows):
    nb = need_backprop.view(-1)
    return nb.long().expand(n_rows) if nb.numel() == 1 else nb.long()


class _ImageDA_drm(nn.Module):
    """lib/MAF/DA.py:128-149: GRL -> DRM -> 1x1 (C*s*s)->512 + ReLU -> 1x1 512->2."""

    def __init__(self, dim, inner_channel, scale):
        super().__init__()
        self.dim = dim
        self.DRM = DRM(dim, inner_channel, scale)
        self.DRM_out = inner_channel * scale * scale
        self.Conv1 = Conv2d(self.DRM_out, 512, 1, bias=False, relu=True)
        self.Conv2 = Conv2d(512, 2, 1, bias=False)

    def forward(self, x, need_backprop):
        x = self.Conv2(self.Conv1(self.DRM(grad_reverse(x))))
        return x, image_label(x, need_backprop)


class _InstanceDA_w(nn.Module):
    """lib/MAF/DA.py:78-104 (no dropout).  need_backprop: the domain label, either one
    value for all rows (the reference) or one per row (source+target batched)."""

    def __init__(self, input):
        super().__init__()
        self.dc_ip1 = Linear(input, 1024)
        self.dc_relu1 = nn.ReLU()
        self.dc_ip2 = Linear(1024, 1024)
        self.dc_relu2 = nn.ReLU()
        self.clssifer = nn.Linear(1024, 2)

    def _mlp(self, x, tap=False):
        h = self.dc_relu1(self.dc_ip1(x))
        if tap and getattr(self.dc_ip1, "act_tap", None) is not None:  # tests
            self.dc_ip1.act_tap.append(h.detach().clone())
        h = self.dc_relu2(self.dc_ip2(h))
        if tap and getattr(self.dc_ip2, "act_tap", None) is not None:
            self.dc_ip2.act_tap.append(h.detach().clone())
        return self.clssifer(h)

    def forward(self, x, need_backprop):
        dom = _row_domain(need_backprop, x.shape[0])
        with torch.no_grad():  # x1 = torch.tensor(x): a detached pass (DA.py:91-94)
            score = F.softmax(self._mlp(x), dim=1)
            w = score.gather(1, dom.view(-1, 1)).view(-1)
        x = self._mlp(wgrad_reverse(x, w), tap=True)
        return x, instance_label_w(x.shape[0], need_backprop.view(-1)[:1])


class _fasterRCNN(_DAFBase):
    """lib/MAF/faster_rcnn.py:22-248 (inherits the DAF detector plumbing)."""

    def __init__(self, classes, class_agnostic):
        super().__init__(classes, class_agnostic)
        del self.RCNN_instanceDA
        del self.consistency_loss
        self.RCNN_imageDA_3 = _ImageDA_drm(256, 64, 4)
        self.RCNN_imageDA_4 = _ImageDA_drm(512, 256, 2)
        self.RCNN_imageDA = _ImageDA(self.dout_base_model)
        self.RCNN_instanceDA = _InstanceDA_w(self.instance_dim + self.n_classes)

    def _backbone(self, im):
        c3 = self.conv3(im)
        c4 = self.conv34(c3)
        return c3, c4, self.conv45(c4)

    @staticmethod
    def _img_loss(score, need):
        return F.nll_loss(F.log_softmax(score, 1), image_label(score, need))

    def forward(self, im_data, im_info, gt_boxes, num_boxes, need_backprop,
                tgt_im_data, tgt_im_info, tgt_gt_boxes, tgt_num_boxes, tgt_need_backprop):
        batch_size = im_data.size(0)
        im_info = im_info.detach()
        gt_boxes = gt_boxes.detach()
        same = (im_data.shape == tgt_im_data.shape) and batch_size == 1
        early = early_rpn(self, same)
        if same:
            c3, c4, base = self._backbone(torch.cat([im_data, tgt_im_data], 0))
            feats = [(c3, c4, base)]
            rpn_in = base.detach().requires_grad_(True) if early else base
            score2, score_r2, prob2, bbox2 = self.RCNN_rpn.head(rpn_in)
            s_score, s_score_r, s_prob, s_bbox = score2[:1], score_r2[:1], prob2[:1], bbox2[:1]
            t_prob, t_bbox = prob2[1:], bbox2[1:]
        else:
            feats = [self._backbone(im_data), self._backbone(tgt_im_data)]
            s_score, s_score_r, s_prob, s_bbox = self.RCNN_rpn.head(feats[0][2])
            _, _, t_prob, t_bbox = self.RCNN_rpn.head(feats[1][2])

        rpn = self.RCNN_rpn
        # proposal layers on side streams, overlapping the anchor target / RPN losses
        pending = proposals_on_side_streams(rpn.RPN_proposal, [
            (s_prob.detach(), s_bbox.detach(), im_info, "TRAIN"),
            (t_prob.detach(), t_bbox.detach(), tgt_im_info.detach(), "TEST")])
        rpn_loss_cls, rpn_loss_bbox, _ = rpn.losses(s_score, s_score_r, s_bbox, gt_boxes, im_info,
                                                    num_boxes, rng=self.replay_rng)
        if early:
            rpn_loss_cls, rpn_loss_bbox = early_rpn_backward(
                rpn_loss_cls, rpn_loss_bbox, rpn_in, [(base, lambda g: g)])
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
            t_rois[:, 0] = 1.0
            feat2 = self._head_to_tail(self._pool(feats[0][2], torch.cat([rois.view(-1, 5), t_rois], 0)))
        else:
            feat2 = torch.cat([self._head_to_tail(self._pool(feats[0][2], rois.view(-1, 5))),
                               self._head_to_tail(self._pool(feats[1][2], tgt_rois.view(-1, 5)))], 0)
        pooled_feat = feat2[:n_s]

        # detection head: one cls_score GEMM over source+target rows (per-row op)
        cls_score2 = self.RCNN_cls_score(feat2)
        cls_prob2 = F.softmax(cls_score2, 1)
        bbox_pred = self.RCNN_bbox_pred(pooled_feat)
        if self.training and not self.class_agnostic:
            view = bbox_pred.view(bbox_pred.size(0), int(bbox_pred.size(1) / 4), 4)
            bbox_pred = torch.gather(view, 1, rois_label.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
        RCNN_loss_cls = F.cross_entropy(cls_score2[:n_s], rois_label)
        from ..detector.losses import smooth_l1_loss
        RCNN_loss_bbox = smooth_l1_loss(bbox_pred, rois_target, rois_inside_ws, rois_outside_ws)
        cls_prob = cls_prob2[:n_s].view(batch_size, n_s, -1)
        bbox_pred = bbox_pred.view(batch_size, n_s, -1)

        # image-level DA on conv3 / conv4 / conv5 (faster_rcnn.py:187-204, 215-235)
        heads = (self.RCNN_imageDA_3, self.RCNN_imageDA_4, self.RCNN_imageDA)
        if same:
            scores = [h(f, need_backprop.new_ones(2))[0] for h, f in zip(heads, feats[0])]
            s_scores, t_scores = [s[:1] for s in scores], [s[1:] for s in scores]
        else:
            s_scores = [h(f, need_backprop)[0] for h, f in zip(heads, feats[0])]
            t_scores = [h(f, tgt_need_backprop)[0] for h, f in zip(heads, feats[1])]
        DA_img_loss_cls = sum(self._img_loss(s, need_backprop) for s in s_scores)
        tgt_DA_img_loss_cls = sum(self._img_loss(s, tgt_need_backprop) for s in t_scores)

        # instance DA on [fc7 || cls_prob] (faster_rcnn.py:206-211, 238-245)
        n_t = feat2.shape[0] - n_s
        dom = torch.cat([need_backprop.view(-1)[:1].long().expand(n_s),
                         tgt_need_backprop.view(-1)[:1].long().expand(n_t)])
        logits, _ = self.RCNN_instanceDA(torch.cat((feat2, cls_prob2), 1), dom)
        y_s = instance_label_w(n_s, need_backprop)
        y_t = instance_label_w(n_t, tgt_need_backprop)
        DA_ins_loss_cls = F.cross_entropy(logits[:n_s], y_s)
        tgt_DA_ins_loss_cls = F.cross_entropy(logits[n_s:], y_t)
        return (rois, cls_prob, bbox_pred, rpn_loss_cls, rpn_loss_bbox, RCNN_loss_cls,
                RCNN_loss_bbox, rois_label, DA_img_loss_cls, DA_ins_loss_cls, tgt_DA_img_loss_cls,
                tgt_DA_ins_loss_cls)

    @staticmethod
    def total_loss(out, lamda=0.1, alpha=1.0):
        """methods/MAF/MAF_train.py:415-418."""
        (_, _, _, rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, _, DA_img, DA_ins,
         tgt_DA_img, tgt_DA_ins) = out
        return weighted_loss_sum(
            (rpn_loss_cls, rpn_loss_box, RCNN_loss_cls, RCNN_loss_bbox, DA_img, DA_ins, tgt_DA_img,
             tgt_DA_ins), (1, 1, 1, 1, lamda, lamda * alpha, lamda, lamda * alpha))


class vgg16(_fasterRCNN):
    """lib/MAF/vgg16.py:20-70: RCNN_base plus the conv3 / conv34 / conv45 views of the
    same modules (features[:16], [16:23], [23:-1])."""

    FUSE_POOLS = (1, 2)  # the DA taps read conv3 / conv4 before pools 3 / 4

    def __init__(self, classes, pretrained=False, class_agnostic=False):
        self.dout_base_model = 512
        self.instance_dim = 4096
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    def _init_modules(self):
        _daf_vgg16._init_modules(self)
        _make_taps(self, VGG16_SPLITS)

    def _head_to_tail(self, pool5):
        return self.RCNN_top(pool5.view(pool5.size(0), -1))


def _make_taps(m, splits):
    _, e3, e4 = splits
    m.conv3, m.conv34, m.conv45 = m.RCNN_base[:e3], m.RCNN_base[e3:e4], m.RCNN_base[e4:]


class resnet(_fasterRCNN):
    """MAF with ResNet101.  lib/MAF/resnet.py builds RCNN_base but not the conv3 / conv34 /
    conv45 taps its forward uses (lib/MAF/faster_rcnn.py:59-61), so it cannot run; built
    here with the taps conv1..layer1 (256 ch) | layer2 (512) | layer3 (1024) — the channel
    counts the MAF discriminators already expect (DRM(256,64,4), DRM(512,256,2)) — and the
    instance head on [2048-d fc7 || cls_prob].  Parity is against the oracle only."""

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
        _make_taps(self, self.RCNN_base.SPLITS)

    train = _daf_resnet.train
    _head_to_tail = _daf_resnet._head_to_tail
    _pool = _daf_resnet._pool
