"""Drop-in ``_RPN`` (lib/model/rpn/rpn.py:17-110) on the tlod kernels.

RPN_Conv (3x3 512->512) + ReLU is one fused libtlod conv; cls/bbox 1x1 convs likewise.
The losses avoid the reference's host syncs (``nonzero`` at :93): cross entropy over
labels != -1 is computed as a masked mean on device, fused with the smooth-L1 box loss into
one forward and one backward launch (tlod_rpn_loss_f32).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import cfg
from ..conv import Conv2d
from ..detector.losses import fused_losses, masked_cross_entropy, rpn_losses, smooth_l1_loss
from .anchor_target import _AnchorTargetLayer
from .proposal import _ProposalLayer


class _RPN(nn.Module):
    def __init__(self, din):
        super().__init__()
        self.din = din
        self.anchor_scales = cfg.ANCHOR_SCALES
        self.anchor_ratios = cfg.ANCHOR_RATIOS
        self.feat_stride = cfg.FEAT_STRIDE[0]
        self.RPN_Conv = Conv2d(self.din, 512, 3, relu=True)
        self.nc_score_out = len(self.anchor_scales) * len(self.anchor_ratios) * 2
        self.RPN_cls_score = Conv2d(512, self.nc_score_out, 1)
        self.nc_bbox_out = len(self.anchor_scales) * len(self.anchor_ratios) * 4
        self.RPN_bbox_pred = Conv2d(512, self.nc_bbox_out, 1)
        self.RPN_proposal = _ProposalLayer(self.feat_stride, self.anchor_scales, self.anchor_ratios)
        self.RPN_anchor_target = _AnchorTargetLayer(self.feat_stride, self.anchor_scales,
                                                    self.anchor_ratios)
        self.rpn_loss_cls = 0
        self.rpn_loss_box = 0

    @staticmethod
    def reshape(x, d):
        s = x.size()
        return x.view(s[0], int(d), int(float(s[1] * s[2]) / float(d)), s[3])

    def head(self, base_feat):
        """conv + scores for a (possibly multi-image) feature batch."""
        rpn_conv1 = self.RPN_Conv(base_feat)
        rpn_cls_score = self.RPN_cls_score(rpn_conv1)
        score_reshape = self.reshape(rpn_cls_score, 2)
        prob = self.reshape(F.softmax(score_reshape, 1), self.nc_score_out)
        bbox = self.RPN_bbox_pred(rpn_conv1)
        return rpn_cls_score, score_reshape, prob, bbox

    def losses(self, rpn_cls_score, score_reshape, bbox, gt_boxes, im_info, num_boxes, rng=None,
               n_images=None):
        """RPN losses of the first ``n_images`` images of a (possibly larger) head batch
        (default: all); the fused path differentiates the whole batch tensors (zero
        gradient for the other images) so no slice enters the autograd graph."""
        B = rpn_cls_score.size(0) if n_images is None else int(n_images)
        labels, targets, inside, outside = self.RPN_anchor_target(
            (rpn_cls_score[:B].detach(), gt_boxes, im_info, num_boxes), rng=rng)
        if fused_losses():
            loss_cls, loss_box = rpn_losses(rpn_cls_score, bbox, labels, targets, inside,
                                            outside, sigma=3.0)
            return loss_cls, loss_box, labels
        score_reshape, bbox = score_reshape[:B], bbox[:B]
        scores = score_reshape.permute(0, 2, 3, 1).contiguous().view(-1, 2)
        loss_cls = masked_cross_entropy(scores, labels.view(B, -1).view(-1))
        loss_box = smooth_l1_loss(bbox, targets, inside, outside, sigma=3, dim=[1, 2, 3])
        return loss_cls, loss_box, labels

    def forward(self, base_feat, im_info, gt_boxes, num_boxes):
        rpn_cls_score, score_reshape, prob, bbox = self.head(base_feat)
        cfg_key = "TRAIN" if self.training else "TEST"
        rois = self.RPN_proposal((prob.detach(), bbox.detach(), im_info, cfg_key))
        self.rpn_loss_cls = 0
        self.rpn_loss_box = 0
        if self.training:
            assert gt_boxes is not None
            self.rpn_loss_cls, self.rpn_loss_box, _ = self.losses(
                rpn_cls_score, score_reshape, bbox, gt_boxes, im_info, num_boxes)
        return rois, self.rpn_loss_cls, self.rpn_loss_box
