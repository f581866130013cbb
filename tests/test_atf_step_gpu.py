"""ATF (lib/ATF) on the device vs the CPU oracle (oracle/atf_step.py): forward losses and
gradients of the two-branch step, same weights (the t branch starts as a copy of the s
branch, vgg16.py:48-50, then both are perturbed so they differ), replayed draws.

Bars: losses within 1e-4 relative; gradients normwise 1e-2 (see test_daf_step_gpu.py).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"

LOSSES = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox", "DA_img_loss_cls",
          "tgt_DA_img_loss_cls", "DA_ins_loss_cls", "tgt_DA_ins_loss_cls"]
IDX = [3, 4, 5, 6, 8, 9, 10, 11]
VIEWS = ("conv3_s.", "conv3_t.", "conv34_s.", "conv34_t.", "conv45_s.", "conv45_t.", "RCNN_rpn_t.")


@pytest.mark.parametrize("net,H,W,seed,ncls", [("vgg16", 192, 320, 0, 9), ("vgg16", 224, 288, 3, 9),
                                               ("res101", 224, 320, 5, 9),
                                               ("res101", 256, 320, 6, 21)])
def test_atf_losses_and_grads_match_oracle(net, H, W, seed, ncls):
    """ncls 21 with ResNet101 (RCNN batch 128, cfgs/res101.yml) is BASELINE config 5's
    detector: ATF ResNet101 PASCAL -> Clipart, the 20 VOC classes + background."""
    from oracle.atf_step import OracleATF, total_loss
    from oracle.daf_step import synthetic_batch
    from tlod.config import cfg
    from tlod.detector.train import build_model
    from tlod.data.imdb import VOC_CLASSES
    from tlod.detector.train import CITYSCAPES_CLASSES
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
    if net == "res101":
        assert o.rcnn_cfg["batch"] == 128 and cfg.TRAIN.BATCH_SIZE == 128
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items() if not k.startswith(VIEWS)}
    o.load_state_dict(sd, strict=True)
    assert cfg.TEST.RPN_POST_NMS_TOP_N == 300
    cpu_batch = synthetic_batch(H, W, seed=seed + 1)
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    out = m(*gpu_batch)
    assert len(out) == 12
    assert cfg.TEST.RPN_POST_NMS_TOP_N == 2000  # the reference's cfg mutation (:260)
    m.total_loss(out).backward()
    cap = m.capture
    ref = o(cpu_batch, np.random.RandomState(3),
            rois_override=tuple(cap[k].cpu().numpy() for k in ("s_rois", "st_rois", "t_rois")))
    total_loss(ref).backward()
    for name, i in zip(LOSSES, IDX):
        g, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    gp = dict(m.named_parameters())
    errs = {}
    for k, p in o.named_parameters():
        if not p.requires_grad:
            continue
        assert gp[k].grad is not None, k
        a, b = gp[k].grad.detach().double().cpu(), p.grad.double()
        errs[k] = float((a - b).norm() / max(b.norm(), 1e-12))
    for k, e in errs.items():
        assert e < 1e-2, (k, e, errs)
    assert all(p.grad is None for p in m.RCNN_rpn_t.parameters())
