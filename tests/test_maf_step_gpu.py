"""MAF (lib/MAF) on the device: the DRM space-to-depth kernels against the literal
chunk/reshape/cat restatement, and the full MAF-VGG16 step (forward losses and gradients)
against the CPU oracle (oracle/maf_step.py) with the same weights and replayed draws.

Bars: space-to-depth / depth-to-space bit-exact (pure permutations); losses within 1e-4
relative; gradients under the pattern-matched fp64 bar (tests/helpers.pattern_grad_bar);
the device's own proposals against the oracle's own as sets (no override).
"""
import numpy as np
import pytest
import torch

from helpers import arm_taps, assert_proposal_sets_match, pattern_grad_bar, record_pattern

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.mark.parametrize("B,C,H,W,s", [(2, 64, 150, 300, 4), (1, 256, 75, 150, 2), (1, 3, 9, 7, 2),
                                       (2, 5, 4, 4, 4), (1, 16, 37, 62, 3)])
def test_space_to_depth_matches_drm_chunks(B, C, H, W, s):
    from oracle.maf_step import drm_chunks
    from tlod.da.maf import space_to_depth
    g = torch.Generator().manual_seed(B * 100 + C + H + W + s)
    x = torch.randn(B, C, H, W, generator=g)
    xd = x.to(dev).requires_grad_(True)
    y = space_to_depth(xd, s)
    ref = drm_chunks(x, s)
    assert torch.equal(y.detach().cpu(), ref)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev))
    xr = x.clone().requires_grad_(True)
    drm_chunks(xr, s).backward(gy)
    assert torch.equal(xd.grad.cpu(), xr.grad)  # cropped border gets exact zeros


def test_wgrl_weights_rows():
    from tlod.da.maf import wgrad_reverse
    x = torch.randn(5, 3, device=dev, requires_grad=True)
    w = torch.tensor([0.1, 0.2, 0.3, 0.4, 0.5], device=dev)
    wgrad_reverse(x, w).sum().backward()
    ref = -0.2 * w.view(-1, 1).expand(5, 3)
    torch.testing.assert_close(x.grad, ref, rtol=0, atol=0)


LOSSES = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox", "DA_img_loss_cls",
          "DA_ins_loss_cls", "tgt_DA_img_loss_cls", "tgt_DA_ins_loss_cls"]
IDX = [3, 4, 5, 6, 8, 9, 10, 11]


def _models(net, H, W, seed):
    from oracle.daf_step import synthetic_batch
    from oracle.maf_step import OracleMAF
    from tlod.detector.train import build_model
    m = build_model("maf", dev, net=net, seed=seed)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    o = OracleMAF(dropout=0.0, backbone=net).train()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()
          if not k.startswith(("conv3.", "conv34.", "conv45."))}  # views of RCNN_base
    o.load_state_dict(sd, strict=True)
    return m, o, synthetic_batch(H, W, seed=seed + 1)


@pytest.mark.parametrize("net,H,W,seed", [("vgg16", 192, 320, 0), ("vgg16", 224, 352, 2),
                                          ("vgg16", 384, 640, 7), ("res101", 224, 320, 4)])
def test_maf_losses_and_grads_match_oracle(net, H, W, seed):
    """Losses 1e-4; sampled RoIs identical; every trainable gradient under the pattern bar
    of the DAF step (tests/helpers.pattern_grad_bar: vs fp64 in the device's activation
    pattern — DRM, the three image discriminators, the weighted-GRL instance MLP, the
    backbone / head ReLUs and max-pools — at most 2x the error of the fp32 references)."""
    from oracle.maf_step import total_loss
    m, o, cpu_batch = _models(net, H, W, seed)
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    taps = arm_taps(m)
    out = m(*gpu_batch)
    assert len(out) == 12
    m.total_loss(out).backward()
    ov = (m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy())
    box = {}

    def run32():
        box["ref"] = o(cpu_batch, np.random.RandomState(3), rois_override=ov)
        total_loss(box["ref"]).backward()
    own = record_pattern(o, run32)
    ref = box["ref"]
    for name, i in zip(LOSSES, IDX):
        g, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    pattern_grad_bar(m, o, lambda mod, b: total_loss(mod(b, np.random.RandomState(3),
                                                         rois_override=ov)),
                     cpu_batch, taps, out[7].numel(), own)


@pytest.mark.parametrize("net,H,W,seed", [("vgg16", 600, 1200, 8), ("res101", 256, 384, 9)])
def test_maf_proposals_without_override(net, H, W, seed):
    """The device's own source (TRAIN) and target (TEST) proposals against the oracle's own
    from each side's RPN outputs (no override), as sets; RPN losses 1e-4."""
    m, o, cpu_batch = _models(net, H, W, seed)
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
