"""End-to-end parity of the DAF-VGG16 step (forward losses and gradients) with the CPU
oracle (oracle/daf_step.py), same weights, dropout off, replayed numpy draws.

The proposal-layer RoIs are taken from the device run (the score sort of near-tied
random-init RPN scores is order-sensitive at the 1e-7 level); everything else —
backbone, RPN losses, anchor/proposal targets, RoIAlign, heads, DA losses — is computed
independently by both sides.  Bar: every loss within 1e-4 relative (north star: 1e-3).
"""
import numpy as np
import pytest
import torch

from helpers import arm_device_taps, assert_proposal_sets_match, pattern_grad_bar, record_pattern

pytestmark = pytest.mark.gpu
dev = "cuda"

LOSSES = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox", "DA_img_loss_cls",
          "DA_ins_loss_cls", "tgt_DA_img_loss_cls", "tgt_DA_ins_loss_cls", "DA_cst_loss",
          "tgt_DA_cst_loss"]
IDX = [3, 4, 5, 6, 8, 9, 10, 11, 12, 13]


def _models(H, W, seed):
    from oracle.daf_step import OracleDAF, synthetic_batch
    from tlod.detector.train import build_daf_vgg16
    m = build_daf_vgg16(dev, seed=seed)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    o = OracleDAF(dropout=0.0).train()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    o.load_state_dict(sd, strict=True)
    cpu_batch = synthetic_batch(H, W, seed=seed + 1)
    return m, o, cpu_batch


@pytest.mark.parametrize("H,W,seed", [(192, 320, 0), (256, 384, 1), (600, 1200, 2)])
def test_daf_losses_and_grads_match_oracle(H, W, seed):
    m, o, cpu_batch = _models(H, W, seed)
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    taps = arm_device_taps(m)
    out = m(*gpu_batch)
    from tlod.detector.train import daf_loss
    loss = daf_loss(out)
    loss.backward()
    ov = (m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy())
    from oracle.daf_step import total_loss
    box = {}

    def run32():
        box["ref"] = o(cpu_batch, np.random.RandomState(3), rois_override=ov)
        total_loss(box["ref"]).backward()
    own = record_pattern(o, run32)
    ref = box["ref"]
    for name, i in zip(LOSSES, IDX):
        g, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    # sampled RoIs identical (replayed draws on identical proposals)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    # gradients of every trainable parameter vs fp64 runs of the same step in matched
    # activation patterns: at most 2x the error of the reference's own fp32 arithmetic
    # (torch CPU, torch on this GPU) — VERDICT r1 2a, tests/helpers.pattern_grad_bar
    pattern_grad_bar(m, o, lambda mod, b: total_loss(mod(b, np.random.RandomState(3),
                                                         rois_override=ov)),
                     cpu_batch, taps, out[7].numel(), own)


@pytest.mark.parametrize("H,W,seed", [(256, 384, 4), (600, 1200, 5)])
def test_daf_proposals_without_override(H, W, seed):
    """the device's own source (TRAIN 12000 -> 2000) and target (TEST 6000 ->
    300) proposals against the oracle's own, from each side's RPN outputs (no override).
    Near-tied random-init scores can reorder the sort and move the top-N boundary, so the
    proposals are compared as sets: >= 99.5% of each side's boxes have an IoU >= 0.999
    partner on the other side.  The RPN losses do not depend on the proposals: 1e-4."""
    m, o, cpu_batch = _models(H, W, seed)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    with torch.no_grad():
        out = m(*tuple(t.to(dev) for t in cpu_batch))
        ref = o._detect(cpu_batch, np.random.RandomState(3))
    for name, i in (("rpn_loss_cls", 3), ("rpn_loss_box", 4)):
        g, r = float(out[i]), float(ref[name])
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    for key, ref_key in (("s_rois", "props"), ("t_rois", "t_props")):
        assert_proposal_sets_match(m.capture[key].cpu().numpy(), ref[ref_key], key)
