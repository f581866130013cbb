"""Source-only Faster R-CNN on the tlod kernels — lib/model/faster_rcnn/{faster_rcnn,vgg16,
resnet}.py, trained by methods/faster_rcnn/faster_rcnn_train.py (BASELINE config 1).

``vgg16(classes).create_architecture()`` then ``model(im_data, im_info, gt_boxes,
num_boxes)`` returns the reference's 8-tuple (faster_rcnn.py:115): rois, cls_prob,
bbox_pred, rpn_loss_cls, rpn_loss_bbox, RCNN_loss_cls, RCNN_loss_bbox, rois_label.  In
eval mode the RPN runs its TEST proposals (6000 -> NMS 0.7 -> 300), the losses are 0 and
bbox_pred keeps every class's deltas (what DAF_test.py / the eval path consume).

Same building blocks as the DAF detector (tlod.da.daf) minus the domain heads: fused
conv + ReLU (+ max-pool) backbone, fused RPN / RCNN losses, device-side anchor / proposal
targets (no host sync), the proposal layer on a side stream while the anchor target and
RPN losses run.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import cfg
from ..roi_align import RoIAlignAvg
from ..roi_pool import _RoIPooling
from ..rpn.proposal import proposals_on_side_streams
from ..rpn.proposal_target import _ProposalTargetLayer
from ..rpn.rpn_head import _RPN
from .losses import fused_losses, rcnn_losses, smooth_l1_loss, weighted_loss_sum
from .vgg16 import vgg16_base, vgg16_top


class _fasterRCNN(nn.Module):
    """lib/model/faster_rcnn/faster_rcnn.py:19-137."""

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
        self.replay_rng = None  # tests: np.random-like object -> reference-exact sampling
        self.capture = None     # tests: dict receiving the proposal-layer rois

    def _pool(self, feat, rois):
        if cfg.POOLING_MODE == "align":
            return self.RCNN_roi_align(feat, rois)
        if cfg.POOLING_MODE == "pool":
            return self.RCNN_roi_pool(feat, rois)
        raise NotImplementedError("POOLING_MODE 'crop' is out of scope (configs use 'align')")

    def forward(self, im_data, im_info, gt_boxes, num_boxes):
        batch_size = im_data.size(0)
        im_info = im_info.detach()
        gt_boxes = gt_boxes.detach()
        base_feat = self.RCNN_base(im_data)
        rpn = self.RCNN_rpn
        score, score_r, prob, bbox = rpn.head(base_feat)
        rpn_loss_cls = rpn_loss_bbox = 0
        rois_label = rois_target = rois_inside_ws = rois_outside_ws = None
        if self.training:
            # rpn.py:74-108: TRAIN proposals on a side stream while this stream does the
            # anchor target and the RPN losses
            pending = proposals_on_side_streams(
                rpn.RPN_proposal, [(prob.detach(), bbox.detach(), im_info, "TRAIN")])
            rpn_loss_cls, rpn_loss_bbox, _ = rpn.losses(score, score_r, bbox, gt_boxes, im_info,
                                                        num_boxes, rng=self.replay_rng)
            (rois,) = pending.join()
            if self.capture is not None:
                self.capture.update(s_rois=rois.detach().clone())
            rois, rois_label, rois_target, rois_inside_ws, rois_outside_ws = \
                self.RCNN_proposal_target(rois, gt_boxes, num_boxes, rng=self.replay_rng)
            rois_label = rois_label.view(-1).long()
            rois_target = rois_target.view(-1, rois_target.size(2))
            rois_inside_ws = rois_inside_ws.view(-1, rois_inside_ws.size(2))
            rois_outside_ws = rois_outside_ws.view(-1, rois_outside_ws.size(2))
        else:
            rois = rpn.RPN_proposal((prob.detach(), bbox.detach(), im_info, "TEST"))

        pooled_feat = self._head_to_tail(self._pool(base_feat, rois.view(-1, 5)))
        bbox_pred = self.RCNN_bbox_pred(pooled_feat)
        RCNN_loss_cls = RCNN_loss_bbox = 0
        if self.training and fused_losses():
            cls_prob, bbox_pred, RCNN_loss_cls, RCNN_loss_bbox = rcnn_losses(
                self.RCNN_cls_score(pooled_feat), bbox_pred, rois_label, rois_target,
                rois_inside_ws, rois_outside_ws, self.class_agnostic)
        else:
            if self.training and not self.class_agnostic:  # faster_rcnn.py:91-95
                view = bbox_pred.view(bbox_pred.size(0), int(bbox_pred.size(1) / 4), 4)
                bbox_pred = torch.gather(view, 1, rois_label.view(-1, 1, 1).expand(-1, 1, 4)
                                         ).squeeze(1)
            cls_score = self.RCNN_cls_score(pooled_feat)
            cls_prob = F.softmax(cls_score, 1)
            if self.training:
                RCNN_loss_cls = F.cross_entropy(cls_score, rois_label)
                RCNN_loss_bbox = smooth_l1_loss(bbox_pred, rois_target, rois_inside_ws,
                                                rois_outside_ws)
        cls_prob = cls_prob.view(batch_size, rois.size(1), -1)
        bbox_pred = bbox_pred.view(batch_size, rois.size(1), -1)
        return (rois, cls_prob, bbox_pred, rpn_loss_cls, rpn_loss_bbox, RCNN_loss_cls,
                RCNN_loss_bbox, rois_label)

    @staticmethod
    def total_loss(out, lamda=None):
        """faster_rcnn_train.py:326-327: the four losses' means, summed."""
        return weighted_loss_sum(out[3:7], (1, 1, 1, 1))

    def _init_weights(self):
        """faster_rcnn.py:117-133 (normal_init, truncated=False)."""
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
    """lib/model/faster_rcnn/vgg16.py:20-66 (random init: the caffe weights are external)."""

    FUSE_POOLS = (1, 2, 3, 4)  # no DA tap reads conv3 / conv4: every max-pool is fused

    def __init__(self, classes, pretrained=False, class_agnostic=False):
        self.dout_base_model = 512
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    def _init_modules(self):
        self.RCNN_base = vgg16_base(fuse_pools=self.FUSE_POOLS)
        self.RCNN_top = vgg16_top()
        self.RCNN_cls_score = nn.Linear(4096, self.n_classes)
        self.RCNN_bbox_pred = nn.Linear(4096, 4 if self.class_agnostic else 4 * self.n_classes)

    def _head_to_tail(self, pool5):
        return self.RCNN_top(pool5.view(pool5.size(0), -1))


class resnet(_fasterRCNN):
    """lib/model/faster_rcnn/resnet.py (ResNet101, frozen BN, layer4 head)."""

    def __init__(self, classes, num_layers=101, pretrained=False, class_agnostic=False):
        if num_layers != 101:
            raise NotImplementedError("only ResNet101 (the configs' depth)")
        self.dout_base_model = 1024
        self.pretrained = pretrained
        self.class_agnostic = class_agnostic
        _fasterRCNN.__init__(self, classes, class_agnostic)

    def _init_modules(self):
        from .resnet import resnet101_parts
        self.RCNN_base, self.RCNN_top = resnet101_parts(cfg.RESNET.FIXED_BLOCKS)
        self.RCNN_cls_score = nn.Linear(2048, self.n_classes)
        self.RCNN_bbox_pred = nn.Linear(2048, 4 if self.class_agnostic else 4 * self.n_classes)

    def train(self, mode=True):
        nn.Module.train(self, mode)
        if mode:
            from .resnet import set_bn_eval
            set_bn_eval(self.RCNN_base)
            set_bn_eval(self.RCNN_top)
        return self

    def _pool(self, feat, rois):
        from .resnet import resnet_pool
        return resnet_pool(self, feat, rois, _fasterRCNN._pool)

    def _head_to_tail(self, pool5):
        return self.RCNN_top(pool5, mean=True)
