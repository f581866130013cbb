"""End-to-end parity of the DAF-VGG16 step (forward losses and gradients) with the CPU
oracle (oracle/daf_step.py), same weights, dropout off, replayed numpy draws.

The proposal-layer RoIs are taken from the device run (the score sort of near-tied
random-init RPN scores is order-sensitive at the 1e-7 level); everything else —
backbone, RPN losses, anchor/proposal targets, RoIAlign, heads, DA losses — is computed
independently by both sides.  Bar: every loss within 1e-4 relative (north star: 1e-3).
"""
import copy

import numpy as np
import pytest
import torch

from helpers import assert_grad_bar, grad_errors

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


@pytest.mark.parametrize("H,W,seed", [(192, 320, 0), (256, 384, 1)])
def test_daf_losses_and_grads_match_oracle(H, W, seed):
    m, o, cpu_batch = _models(H, W, seed)
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    out = m(*gpu_batch)
    from tlod.detector.train import daf_loss
    loss = daf_loss(out)
    loss.backward()
    ref = o(cpu_batch, np.random.RandomState(3),
            rois_override=(m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy()))
    from oracle.daf_step import total_loss
    rl = total_loss(ref)
    rl.backward()
    for name, i in zip(LOSSES, IDX):
        g, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    # sampled RoIs identical (replayed draws on identical proposals)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    # gradients of every trainable parameter against an fp64 run of the same step (same
    # weights, RoIs and draws): at most 2x the fp32 CPU oracle's own error
    o64 = copy.deepcopy(o).double()
    for p in o64.parameters():
        p.grad = None
    b64 = tuple(t.double() if t.is_floating_point() else t for t in cpu_batch)
    r64 = o64(b64, np.random.RandomState(3),
              rois_override=(m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy()))
    total_loss(r64).backward()
    errs = grad_errors(m.named_parameters(), o, o64)
    print({k: (f"{a:.2e}", f"{b:.2e}") for k, (a, b) in errs.items()})
    assert_grad_bar(errs)
