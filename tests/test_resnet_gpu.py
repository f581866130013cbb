"""ResNet101 on the device (tlod.detector.resnet) vs the torch-CPU restatement
(oracle/resnet.py) with identical weights: the stem kernel, the stride-2 subsample pair,
the fused conv+BN(+residual)+ReLU epilogue, whole bottlenecks (NCHW backbone path and the
channels-last RoI-head path), and the DAF-ResNet101 training step against the oracle.

Bars: permutations bit-exact; fp32 conv arithmetic normwise 1e-5 per layer (the MFMA path
is an exact-f32 FMA chain); full-step losses 1e-4 relative, gradients under the
pattern-matched fp64 bar (tests/helpers.pattern_grad_bar), proposals as sets.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _close(got, ref, tol=1e-5):
    got, ref = got.detach().double().cpu(), ref.detach().double().cpu()
    err = float((got - ref).norm() / max(float(ref.norm()), 1e-30))
    assert err <= tol, err


def _rand_bn(bn, g):
    with torch.no_grad():
        bn.weight.copy_(torch.rand(bn.weight.shape, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(bn.bias.shape, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(bn.running_mean.shape, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(bn.running_var.shape, generator=g) + 0.5)


@pytest.mark.parametrize("H,W", [(64, 96), (37, 51)])
def test_stem_conv(H, W):
    from tlod.detector.resnet import stem
    g = torch.Generator().manual_seed(H + W)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False)
    bn = torch.nn.BatchNorm2d(64).eval()
    _rand_bn(bn, g)
    for p in list(conv.parameters()) + list(bn.parameters()):
        p.requires_grad = False
    x = torch.randn(2, 3, H, W, generator=g) * 50
    ref = F.relu(bn(conv(x)))
    got = stem(x.to(dev), conv.to(dev), bn.to(dev))
    assert got.shape == ref.shape
    _close(got, ref)


@pytest.mark.parametrize("H,W", [(8, 10), (7, 7), (38, 75)])
def test_subsample_pair_exact(H, W):
    from tlod.detector.resnet import Subsample2Function
    x = torch.randn(2, 3, H, W, device=dev, requires_grad=True)
    y = Subsample2Function.apply(x)
    assert torch.equal(y, x[:, :, ::2, ::2])
    gy = torch.randn_like(y)
    y.backward(gy)
    ref = torch.zeros_like(x)
    ref[:, :, ::2, ::2] = gy
    assert torch.equal(x.grad, ref)


@pytest.mark.parametrize("KS,res", [(1, True), (3, False), (3, True)])
def test_conv_bn_epilogue(KS, res):
    from tlod.conv import ConvBNFunction
    g = torch.Generator().manual_seed(KS * 10 + res)
    x = torch.randn(2, 64, 19, 37, generator=g)
    w = torch.randn(128, 64, KS, KS, generator=g) * 0.05
    sc, sh = torch.rand(128, generator=g) + 0.5, torch.randn(128, generator=g)
    r = torch.randn(2, 128, 19, 37, generator=g) if res else None
    xd, wd = x.to(dev).requires_grad_(True), w.to(dev).requires_grad_(True)
    rd = r.to(dev).requires_grad_(True) if res else None
    y = ConvBNFunction.apply(xd, wd, sc.to(dev), sh.to(dev), rd, True)
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    rr = r.double().requires_grad_(True) if res else None
    pre = F.conv2d(xr, wr, padding=KS // 2) * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
    if res:
        pre = pre + rr
    _close(y, F.relu(pre))
    yr = pre * (y.detach().cpu() > 0).double()  # backward through the device's mask
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev))
    yr.backward(gy.double())
    _close(xd.grad, xr.grad)
    _close(wd.grad, wr.grad)
    if res:
        _close(rd.grad, rr.grad)


def _pair_blocks(inplanes, planes, stride, seed):
    from oracle.resnet import Bottleneck as OB
    from tlod.detector.resnet import Bottleneck
    g = torch.Generator().manual_seed(seed)
    ds = None
    if stride != 1 or inplanes != planes * 4:
        ds = torch.nn.Sequential(torch.nn.Conv2d(inplanes, planes * 4, 1, stride, bias=False),
                                 torch.nn.BatchNorm2d(planes * 4))
    ob = OB(inplanes, planes, stride, ds).eval()
    for m in ob.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            _rand_bn(m, g)
            for p in m.parameters():
                p.requires_grad = False
        elif isinstance(m, torch.nn.Conv2d):
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / m.weight[0].numel()) ** 0.5)
    ds2 = None
    if ds is not None:
        ds2 = torch.nn.Sequential(torch.nn.Conv2d(inplanes, planes * 4, 1, stride, bias=False),
                                  torch.nn.BatchNorm2d(planes * 4))
    db = Bottleneck(inplanes, planes, stride, ds2)
    db.load_state_dict(ob.state_dict())
    for m in db.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            for p in m.parameters():
                p.requires_grad = False
    return ob, db.to(dev).eval(), g


@pytest.mark.parametrize("inplanes,planes,stride,H,W", [(256, 64, 1, 20, 36), (256, 128, 2, 19, 37),
                                                        (512, 128, 1, 10, 19)])
def test_bottleneck_nchw(inplanes, planes, stride, H, W):
    ob, db, g = _pair_blocks(inplanes, planes, stride, inplanes + planes + stride)
    x = torch.randn(2, inplanes, H, W, generator=g)
    xd = x.to(dev).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y, yr = db(xd), ob(xr)
    _close(y, yr, 1e-5)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev))
    yr.backward(gy)
    _close(xd.grad, xr.grad, 1e-4)
    for (k, p), (_, q) in zip(db.named_parameters(), ob.named_parameters()):
        if q.requires_grad:
            _close(p.grad, q.grad, 1e-4)


@pytest.mark.parametrize("inplanes,planes,stride,R", [(1024, 512, 2, 6), (2048, 512, 1, 5)])
def test_bottleneck_head_nhwc(inplanes, planes, stride, R):
    ob, db, g = _pair_blocks(inplanes, planes, stride, R)
    H = 7 if stride == 2 else 4
    x = torch.randn(R, inplanes, H, H, generator=g)
    xd = x.to(dev).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y2, shp = db.forward_nhwc(xd.permute(0, 2, 3, 1))
    y = y2.view(*shp, -1).permute(0, 3, 1, 2)
    yr = ob(xr)
    _close(y, yr, 1e-5)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev))
    yr.backward(gy)
    _close(xd.grad, xr.grad, 1e-4)


@pytest.mark.parametrize("R,entry", [(37, True), (5, False)])
def test_head_fused_backward_bit_identical(R, entry, monkeypatch):
    """The RoI head's fused backward (TLOD_HEAD_FUSE=1: each ReLU mask in the consumer's
    input-gradient epilogue — tlod_gemm_bs_mask_f32, tlod_col2im3x3_nhwc_mask_f32 — and the
    identity shortcut's gradient added in conv1's input-gradient GEMM) against the unfused
    chain (torch.where masks, autograd's sum), over layer4's three bottlenecks: output, input
    gradient and every weight / bias gradient bit for bit.  entry: the head-entry input
    (already subsampled, 4x4) or the 7x7 map."""
    from tlod import linear
    from tlod.detector.resnet import ResNetTop, HeadEntry, _make_layer
    g = torch.Generator().manual_seed(R)
    layer = _make_layer(1024, 512, 3, stride=2)
    for m in layer.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            _rand_bn(m, g)
            for p in m.parameters():
                p.requires_grad = False
        elif isinstance(m, torch.nn.Conv2d):
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / m.weight[0].numel()) ** 0.5)
    top = ResNetTop(layer).to(dev)
    H = 4 if entry else 7
    x = torch.randn(R, H, H, 1024, generator=g).to(dev)
    gy = torch.randn(R, 2048, generator=g).to(dev)

    def run(fuse, implicit="0"):
        monkeypatch.setenv("TLOD_HEAD_FUSE", fuse)
        monkeypatch.setenv("TLOD_HEAD_IMPLICIT", implicit)
        for p in top.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        y = top(HeadEntry(xi) if entry else xi.permute(0, 3, 1, 2))
        (y.mean(2).mean(1) * gy).sum().backward()
        return [y.detach(), xi.grad] + [p.grad for p in top.parameters() if p.requires_grad]
    before = dict(linear.STATS)
    fused = run("1")
    assert linear.STATS["masked_dgrad"] - before["masked_dgrad"] == 5  # 3 x conv3 + 2 x conv1
    assert linear.STATS["relu_bwd_skipped"] - before["relu_bwd_skipped"] == 8  # + 3 x conv1 (col2im)
    plain = run("0")
    for i, (a, b) in enumerate(zip(fused, plain)):
        assert torch.equal(a, b), i
    # round 6: conv2 as implicit GEMMs over the map (the default).  The forward and conv2's
    # weight gradient take the same K order as the im2col GEMMs: bit for bit; the input
    # gradient sums its 9 x 512 products in one GEMM instead of a GEMM + col2im's 9-tap sum,
    # so every gradient upstream of it agrees to f32 rounding
    before = dict(linear.STATS)
    impl = run("1", "1")
    assert linear.STATS["masked_dgrad"] - before["masked_dgrad"] == 8  # + 3 x conv2's input grad
    assert linear.STATS["relu_bwd_skipped"] - before["relu_bwd_skipped"] == 8
    assert torch.equal(impl[0], plain[0])
    for i, (a, b) in enumerate(zip(impl[1:], plain[1:])):
        err = float((a.double() - b.double()).norm() / b.double().norm())
        assert err < 1e-5, (i, err)


@pytest.mark.parametrize("entry", [True, False])
def test_head_mean_in_last_gemm_bit_identical(entry):
    """fc7 = RCNN_top(pool5).mean(3).mean(2) taken inside the last conv3's GEMM function
    (ResNetTop(..., mean=True) -> LinearActFunction mean_hw) against head_mean over the
    channels-last output: fc7, the input gradient and every weight gradient bit for bit."""
    from tlod.detector.resnet import ResNetTop, HeadEntry, _make_layer, head_mean
    g = torch.Generator().manual_seed(11)
    layer = _make_layer(1024, 512, 3, stride=2)
    for m in layer.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            _rand_bn(m, g)
            for p in m.parameters():
                p.requires_grad = False
        elif isinstance(m, torch.nn.Conv2d):
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / m.weight[0].numel()) ** 0.5)
    top = ResNetTop(layer).to(dev)
    R, H = 37, 4 if entry else 7
    x = torch.randn(R, H, H, 1024, generator=g).to(dev)
    gy = torch.randn(R, 2048, generator=g).to(dev)

    def run(fused):
        for p in top.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        inp = HeadEntry(xi) if entry else xi.permute(0, 3, 1, 2)
        f = top(inp, mean=True) if fused else head_mean(top(inp))
        assert f.shape == (R, 2048)
        (f * gy).sum().backward()
        return [f.detach(), xi.grad] + [p.grad for p in top.parameters() if p.requires_grad]
    a, b = run(True), run(False)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), i


LOSSES = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox", "DA_img_loss_cls",
          "DA_ins_loss_cls", "tgt_DA_img_loss_cls", "tgt_DA_ins_loss_cls", "DA_cst_loss",
          "tgt_DA_cst_loss"]
IDX = [3, 4, 5, 6, 8, 9, 10, 11, 12, 13]


def _daf_r101(seed, H, W):
    from oracle.daf_step import OracleDAF, synthetic_batch
    from tlod.detector.train import build_model
    m = build_model("daf", dev, net="res101", seed=seed)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    o = OracleDAF(dropout=0.0, backbone="res101").train()
    o.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=True)
    return m, o, synthetic_batch(H, W, seed=seed + 1)


@pytest.mark.parametrize("H,W,seed", [(224, 320, 5), (320, 512, 7)])
def test_daf_resnet101_step_matches_oracle(H, W, seed):
    """BASELINE config 3's detector: losses 1e-4, sampled RoIs identical, every trainable
    gradient (layer2 / layer3 bottlenecks, the layer4 RoI head, RPN, DA heads) under the
    pattern-matched fp64 bar (tests/helpers.pattern_grad_bar)."""
    from oracle.daf_step import total_loss
    from helpers import arm_taps, pattern_grad_bar, record_pattern
    m, o, cpu_batch = _daf_r101(seed, H, W)
    gpu_batch = tuple(t.to(dev) for t in cpu_batch)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    taps = arm_taps(m)
    out = m(*gpu_batch)
    m.total_loss(out).backward()
    assert out[0].shape[1] == 128  # cfgs/res101.yml TRAIN.BATCH_SIZE
    ov = (m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy())
    box = {}

    def run32():
        box["ref"] = o(cpu_batch, np.random.RandomState(3), rois_override=ov)
        total_loss(box["ref"]).backward()
    own = record_pattern(o, run32)
    ref = box["ref"]
    for name, i in zip(LOSSES, IDX):
        gv, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(gv - r) <= 1e-4 * max(abs(r), 1e-3), (name, gv, r)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    pattern_grad_bar(m, o, lambda mod, b: total_loss(mod(b, np.random.RandomState(3),
                                                         rois_override=ov)),
                     cpu_batch, taps, out[7].numel(), own)


def test_daf_resnet101_proposals_without_override():
    from helpers import assert_proposal_sets_match
    m, o, cpu_batch = _daf_r101(13, 320, 640)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    with torch.no_grad():
        out = m(*tuple(t.to(dev) for t in cpu_batch))
        ref = o._detect(cpu_batch, np.random.RandomState(3))
    for name, i in (("rpn_loss_cls", 3), ("rpn_loss_box", 4)):
        gv, r = float(out[i]), float(ref[name])
        assert abs(gv - r) <= 1e-4 * max(abs(r), 1e-3), (name, gv, r)
    for key, ref_key in (("s_rois", "props"), ("t_rois", "t_props")):
        assert_proposal_sets_match(m.capture[key].cpu().numpy(), ref[ref_key], key)


@pytest.mark.parametrize("R,H,W,C", [(5, 4, 4, 32), (3, 2, 7, 512), (2, 1, 1, 4)])
def test_im2col3x3_nhwc(R, H, W, C):
    """tlod_im2col3x3_nhwc_f32 / col2im (the RoI head's 3x3 convs) against the torch
    composition they replace (F.pad + 9 slices + cat): forward bit-exact, backward to fp32
    summation order."""
    import torch.nn.functional as F
    from tlod.detector.resnet import Im2col3x3Function
    g = torch.Generator().manual_seed(R * 100 + C)
    x = torch.randn(R, H, W, C, generator=g).to(dev).requires_grad_(True)
    col = Im2col3x3Function.apply(x)
    xr = x.detach().clone().requires_grad_(True)
    pad = F.pad(xr, (0, 0, 1, 1, 1, 1))
    ref = torch.cat([pad[:, kh:kh + H, kw:kw + W, :] for kh in range(3) for kw in range(3)],
                    3).reshape(R * H * W, 9 * C)
    assert torch.equal(col, ref)
    gy = torch.randn(R * H * W, 9 * C, generator=g).to(dev)
    col.backward(gy)
    ref.backward(gy)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-6, atol=1e-6)
