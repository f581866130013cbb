"""ATF (lib/ATF) on the device vs the CPU oracle (oracle/atf_step.py): forward losses and
gradients of the two-branch step, same weights (the t branch starts as a copy of the s
branch, vgg16.py:48-50, then both are perturbed so they differ), replayed draws.

Bars: losses within 1e-4 relative; gradients under the pattern-matched fp64 bar
(tests/helpers.pattern_grad_bar: both backbones, the three RPN passes, the four RoI sets
through the head, the image and instance discriminators); the device's own s-branch,
t-branch and target proposals against the oracle's own, as sets (no override).
"""
import numpy as np
import pytest
import torch

from helpers import arm_taps, assert_proposal_sets_match, pattern_grad_bar, record_pattern

pytestmark = pytest.mark.gpu
dev = "cuda"

LOSSES = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox", "DA_img_loss_cls",
          "tgt_DA_img_loss_cls", "DA_ins_loss_cls", "tgt_DA_ins_loss_cls"]
IDX = [3, 4, 5, 6, 8, 9, 10, 11]
VIEWS = ("conv3_s.", "conv3_t.", "conv34_s.", "conv34_t.", "conv45_s.", "conv45_t.", "RCNN_rpn_t.")


def _models(net, H, W, seed, ncls):
    from oracle.atf_step import OracleATF
    from oracle.daf_step import synthetic_batch
    from tlod.data.imdb import VOC_CLASSES
    from tlod.detector.train import CITYSCAPES_CLASSES, build_model
    classes = VOC_CLASSES if ncls == 21 else CITYSCAPES_CLASSES
    m = build_model("atf", dev, net=net, seed=seed, classes=classes)
    with torch.no_grad():  # make the two branches differ
        for p in m.RCNN_base_t[m.splits[0]:].parameters():
            if p.requires_grad:
                p.mul_(1.0 + 0.05 * torch.randn_like(p))
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    o = OracleATF(n_classes=ncls, dropout=0.0, backbone=net).train()
    assert m.RCNN_cls_score.out_features == ncls
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items() if not k.startswith(VIEWS)}
    o.load_state_dict(sd, strict=True)
    return m, o, synthetic_batch(H, W, seed=seed + 1)


@pytest.mark.parametrize("net,H,W,seed,ncls", [("vgg16", 192, 320, 0, 9), ("vgg16", 224, 288, 3, 9),
                                               ("vgg16", 320, 512, 7, 9),
                                               ("res101", 224, 320, 5, 9),
                                               ("res101", 256, 320, 6, 21)])
def test_atf_losses_and_grads_match_oracle(net, H, W, seed, ncls):
    """ncls 21 with ResNet101 (RCNN batch 128, cfgs/res101.yml) is BASELINE config 5's
    detector: ATF ResNet101 PASCAL -> Clipart, the 20 VOC classes + background."""
    from oracle.atf_step import total_loss
    from tlod.config import cfg
    m, o, cpu_batch = _models(net, H, W, seed, ncls)
    if net == "res101":
        assert o.rcnn_cfg["batch"] == 128 and cfg.TRAIN.BATCH_SIZE == 128
    assert cfg.TEST.RPN_POST_NMS_TOP_N == 300
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    taps = arm_taps(m)
    out = m(*gpu_batch)
    assert len(out) == 12
    assert cfg.TEST.RPN_POST_NMS_TOP_N == 2000  # the reference's cfg mutation (:260)
    m.total_loss(out).backward()
    cap = m.capture
    ov = tuple(cap[k].cpu().numpy() for k in ("s_rois", "st_rois", "t_rois"))
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
    gp = dict(m.named_parameters())
    for k, p in o.named_parameters():
        if p.requires_grad:
            assert gp[k].grad is not None, k
    assert all(p.grad is None for p in m.RCNN_rpn_t.parameters())
    # head rows: s-branch sampled, t-branch sampled, t-branch proposals, target proposals
    nb = out[7].numel()
    rows = {"head": [nb, nb, ov[1].shape[1], ov[2].shape[1]], "ins": [ov[1].shape[1], ov[2].shape[1]]}
    pattern_grad_bar(m, o, lambda mod, b: total_loss(mod(b, np.random.RandomState(3),
                                                         rois_override=ov)),
                     cpu_batch, taps, rows, own)


@pytest.mark.parametrize("net,H,W,seed", [("vgg16", 384, 768, 11), ("res101", 256, 384, 12)])
def test_atf_proposals_without_override(net, H, W, seed):
    """ATF's three proposal passes (lib/ATF/faster_rcnn.py:130-134, 258-262): the s and t
    branches on the source image (TRAIN, 12000 -> 2000) and the target image (TEST with
    post-NMS top-N mutated to 2000), each from the side's own RPN outputs; RPN losses
    (summed over both branches) 1e-4."""
    m, o, cpu_batch = _models(net, H, W, seed, 9)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    with torch.no_grad():
        out = m(*tuple(t.to(dev) for t in cpu_batch))
        ref = o(cpu_batch, np.random.RandomState(3))
    for name, i in (("rpn_loss_cls", 3), ("rpn_loss_box", 4)):
        g, r = float(out[i]), float(ref[name])
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    for key, ref_key in (("s_rois", "props_s"), ("st_rois", "props_st"), ("t_rois", "props_t")):
        assert_proposal_sets_match(m.capture[key].cpu().numpy(), ref[ref_key], key)
