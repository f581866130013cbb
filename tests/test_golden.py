"""Golden fixtures (tests/golden/golden_v1.npz, made by make_golden.py from the oracle).

CPU: the oracle still reproduces every fixture (guards the restatement against drift).
GPU: the HIP path reproduces them through the C ABI (same bars as the parity tests)."""
import os

import numpy as np
import pytest
import torch

from oracle import nms as onms
from oracle import roi as oroi
from oracle import rpn as orpn
from oracle.boxes import generate_anchors

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))


class Replay:
    """Replays recorded np.random draws (kind 0 = permutation, 1 = rand) in order."""

    def __init__(self, prefix):
        self.kinds = G[prefix + "_draw_kinds"]
        self.lens = G[prefix + "_draw_lens"]
        self.flat = G[prefix + "_draws"]
        self.i, self.off = 0, 0

    def _next(self, kind, n):
        assert self.kinds[self.i] == kind and self.lens[self.i] == n
        v = self.flat[self.off:self.off + n]
        self.i += 1
        self.off += n
        return v

    def permutation(self, n):
        return self._next(0, n).astype(np.int64)

    def rand(self, n):
        return self._next(1, n)


def test_oracle_reproduces_golden():
    base = generate_anchors(scales=np.array([4, 8, 16, 32]), ratios=np.array([0.5, 1, 2]))
    np.testing.assert_array_equal(base, G["anchors_base"])
    np.testing.assert_array_equal(onms.nms(G["nms_dets"], 0.7), G["nms_keep_07"])
    np.testing.assert_array_equal(onms.nms(G["nms_dets"], 0.3), G["nms_keep_03"])
    f, r = G["roi_feat"], G["roi_rois"]
    np.testing.assert_array_equal(oroi.roi_align_fwd(f, r, 8, 8, 1 / 16), G["roi_align8"])
    np.testing.assert_array_equal(oroi.roi_align_avg_fwd(f, r, 7, 7, 1 / 16), G["roi_align_avg"])
    np.testing.assert_allclose(oroi.roi_align_avg_bwd(G["roi_g7"], r, 1, 8, 12, 16, 1 / 16),
                               G["roi_align_avg_bwd"], rtol=1e-6, atol=1e-7)
    po, pa = oroi.roi_pool_fwd(f, r, 7, 7, 1 / 16)
    np.testing.assert_array_equal(po, G["roi_pool"])
    np.testing.assert_array_equal(pa, G["roi_pool_argmax"])
    rois = orpn.proposal_layer(G["prop_prob"], G["prop_deltas"], G["prop_info"], base, 16, 1000,
                               200, 0.7)
    np.testing.assert_array_equal(rois, G["prop_rois"])
    at = orpn.anchor_target(10, 12, G["at_gt"], G["prop_info"], base, 16, Replay("at"))
    for k, v in zip(["at_labels", "at_targets", "at_inside", "at_outside"], at):
        np.testing.assert_array_equal(v, G[k])
    pt = orpn.proposal_target(G["pt_rois_in"], G["at_gt"], Replay("pt"))
    for k, v in zip(["pt_rois", "pt_labels", "pt_targets", "pt_inside", "pt_outside"], pt):
        np.testing.assert_array_equal(v, G[k])


@pytest.mark.gpu
def test_hip_reproduces_golden():
    from tlod.nms import nms
    from tlod.roi_align import RoIAlignAvg, RoIAlignFunction
    from tlod.roi_pool import roi_pool_with_argmax
    from tlod.rpn.anchor_target import anchor_target, rpn_cfg_struct
    from tlod.rpn.proposal import proposal
    from tlod.rpn.proposal_target import proposal_target, rcnn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    t = lambda k: torch.from_numpy(np.ascontiguousarray(G[k])).cuda()
    np.testing.assert_array_equal(nms(t("nms_dets"), 0.7).cpu().numpy(), G["nms_keep_07"])
    np.testing.assert_array_equal(nms(t("nms_dets"), 0.3).cpu().numpy(), G["nms_keep_03"])
    f = t("roi_feat").requires_grad_(True)
    np.testing.assert_array_equal(RoIAlignFunction.apply(f, t("roi_rois"), 8, 8, 1 / 16)
                                  .detach().cpu().numpy(), G["roi_align8"])
    o = RoIAlignAvg(7, 7, 1 / 16)(f, t("roi_rois"))
    np.testing.assert_array_equal(o.detach().cpu().numpy(), G["roi_align_avg"])
    o.backward(t("roi_g7"))
    np.testing.assert_allclose(f.grad.cpu().numpy(), G["roi_align_avg_bwd"], rtol=1e-5, atol=1e-6)
    f2 = t("roi_feat").requires_grad_(True)
    po, pa = roi_pool_with_argmax(f2, t("roi_rois"), 7, 7, 1 / 16)
    np.testing.assert_array_equal(po.detach().cpu().numpy(), G["roi_pool"])
    np.testing.assert_array_equal(pa.cpu().numpy(), G["roi_pool_argmax"])
    po.backward(t("roi_g7"))
    np.testing.assert_allclose(f2.grad.cpu().numpy(), G["roi_pool_bwd"], rtol=1e-5, atol=1e-6)
    rois = proposal(t("prop_prob"), t("prop_deltas"), t("prop_info"), t("anchors_base"), 16,
                    1000, 200, 0.7)
    np.testing.assert_array_equal(rois.cpu().numpy(), G["prop_rois"])  # deltas 0: exact decode
    at = anchor_target(t("anchors_base"), 10, 12, 16, t("at_gt"), t("prop_info"), rpn_cfg_struct(),
                       rng=Replay("at"))
    for k, v in zip(["at_labels", "at_targets", "at_inside", "at_outside"], at):
        np.testing.assert_allclose(v.cpu().numpy(), G[k], rtol=2e-6, atol=2e-6, err_msg=k)
    pt = proposal_target(t("pt_rois_in"), t("at_gt"), rcnn_cfg_struct(), rng=Replay("pt"))
    for k, v in zip(["pt_rois", "pt_labels", "pt_targets", "pt_inside", "pt_outside"], pt):
        np.testing.assert_allclose(v.cpu().numpy(), G[k], rtol=2e-6, atol=2e-6, err_msg=k)
