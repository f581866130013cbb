"""Regenerate the golden fixtures in this directory from the oracle restatement.

    python tests/golden/make_golden.py

Inputs are seeded synthetic tensors of the reference's shapes; outputs come from the
CPU restatement (oracle/), whose anchor generator is pinned by the reference's own
known-answer table (generate_anchors.py:29-37).  The fixtures freeze the restatement so
both the oracle (tests/test_golden.py, CPU) and the HIP path (GPU) are checked against
the same vectors; recorded numpy draws let the HIP targets replay the sampling.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import clustered_boxes, gt_set, rpn_outputs, sorted_dets  # noqa: E402
from oracle import nms as onms  # noqa: E402
from oracle import roi as oroi  # noqa: E402
from oracle import rpn as orpn  # noqa: E402
from oracle.boxes import generate_anchors  # noqa: E402


def draws_to_arrays(log):
    kinds = np.array([0 if k == "perm" else 1 for k, _ in log], np.int8)
    lens = np.array([len(x) for _, x in log], np.int64)
    flat = np.concatenate([np.asarray(x, np.float64) for _, x in log]) if log else np.zeros(0)
    return kinds, lens, flat


def main():
    out = {}
    base = generate_anchors(scales=np.array([4, 8, 16, 32]), ratios=np.array([0.5, 1, 2]))
    out["anchors_base"] = base

    rng = np.random.default_rng(2024)
    d = sorted_dets(clustered_boxes(rng, 700, clusters=60), rng)
    out["nms_dets"] = d
    out["nms_keep_07"] = onms.nms(d, 0.7)
    out["nms_keep_03"] = onms.nms(d, 0.3)

    feat = rng.standard_normal((1, 8, 12, 16)).astype(np.float32)
    rois = np.zeros((10, 5), np.float32)
    rois[:, 1:3] = rng.uniform(-20, 180, (10, 2))
    rois[:, 3:5] = rois[:, 1:3] + rng.uniform(-5, 150, (10, 2))
    g7 = rng.standard_normal((10, 8, 7, 7)).astype(np.float32)
    out["roi_feat"], out["roi_rois"], out["roi_g7"] = feat, rois, g7
    out["roi_align8"] = oroi.roi_align_fwd(feat, rois, 8, 8, 1 / 16)
    out["roi_align_avg"] = oroi.roi_align_avg_fwd(feat, rois, 7, 7, 1 / 16)
    out["roi_align_avg_bwd"] = oroi.roi_align_avg_bwd(g7, rois, 1, 8, 12, 16, 1 / 16)
    po, pa = oroi.roi_pool_fwd(feat, rois, 7, 7, 1 / 16)
    out["roi_pool"], out["roi_pool_argmax"] = po, pa
    out["roi_pool_bwd"] = oroi.roi_pool_bwd(g7, pa, rois, 1, 8, 12, 16, 1 / 16)

    A, H, W = 12, 10, 12
    prob, deltas = rpn_outputs(rng, 1, A, H, W, delta_scale=0.0)
    info = np.array([[H * 16, W * 16, 1.0]], np.float32)
    out["prop_prob"], out["prop_deltas"], out["prop_info"] = prob, deltas, info
    out["prop_rois"] = orpn.proposal_layer(prob, deltas, info, base, 16, 1000, 200, 0.7)

    gts = gt_set(rng, G=5, pad=20, W=W * 16, H=H * 16)[None]
    rec = orpn.Recorder(5)
    lab, tgt, iw, ow = orpn.anchor_target(H, W, gts, info, base, 16, rec)
    out["at_gt"] = gts
    out["at_labels"], out["at_targets"], out["at_inside"], out["at_outside"] = lab, tgt, iw, ow
    out["at_draw_kinds"], out["at_draw_lens"], out["at_draws"] = draws_to_arrays(rec.log)

    pr = np.zeros((1, 200, 5), np.float32)
    near = gts[0, rng.integers(0, 5, 100), :4] + rng.normal(0, 6, (100, 4))
    far = rng.uniform(0, 180, (90, 4))
    far[:, 2:] = far[:, :2] + rng.uniform(4, 60, (90, 2))
    pr[0, :190, 1:] = np.clip(np.concatenate([near, far]), 0, 191).astype(np.float32)
    rec = orpn.Recorder(6)
    res = orpn.proposal_target(pr, gts, rec)
    out["pt_rois_in"] = pr
    for k, v in zip(["pt_rois", "pt_labels", "pt_targets", "pt_inside", "pt_outside"], res):
        out[k] = v
    out["pt_draw_kinds"], out["pt_draw_lens"], out["pt_draws"] = draws_to_arrays(rec.log)

    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
