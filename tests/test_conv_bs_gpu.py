"""Split-bf16 3x3 convolution (tlod_conv_fwd_bs_f32: f32 operands split exactly into three
bf16 terms, products on the bf16 MFMA, f32 accumulation) vs a PyTorch fp64 CPU reference.

Bars (normwise relative / elementwise vs max|ref|): bf16x6 — the same 1e-5 / 1e-4 bar as
the f32-input MFMA path (measured error is f32-rounding level); bf16x3 — 5e-5 / 5e-4
(dropped terms are ~2^-16 relative per product).  Forward (with the BN-fold / residual /
ReLU epilogue) and dgrad, including the split-K tail schedule and ragged channel counts.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
BARS = {"bf16x6": (1e-5, 1e-4), "bf16x3": (5e-5, 5e-4)}


def _close(got, ref, math):
    tol, etol = BARS[math]
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    nrm = float((got - ref).norm() / max(float(ref.norm()), 1e-30))
    assert nrm <= tol, f"{math}: normwise rel err {nrm:.3e}"
    assert float((got - ref).abs().max()) <= etol * float(ref.abs().max()) + 1e-30
    return nrm


SHAPES = [  # N, Cin, Cout, H, W
    (2, 64, 128, 37, 75), (1, 3, 64, 50, 70), (2, 256, 256, 30, 40), (1, 512, 512, 37, 62),
    (1, 13, 20, 9, 33), (1, 130, 132, 9, 33), (1, 64, 256, 150, 250),
    # warp-specialized kernel (Cin >= 128) on its run-time tiles (ws_tile): 15 x 34 at
    # 150 x 300, 13 x 39 at 75 x 150, 19 x 26 at 37 x 75, 2 x 158 rows, blocks wrapping rows
    (2, 256, 256, 150, 300), (1, 128, 136, 75, 150), (1, 256, 64, 37, 75), (1, 128, 128, 2, 700),
    (1, 144, 128, 61, 9),
    # round 5 staging layout: 30 x 17 tiles (row pitch TW + 16) at 150 x 250, 4 x 125 at 75 x 125
    (1, 128, 136, 150, 250), (1, 136, 128, 75, 125),
    # stream-K tail (plan_stream_k: conv5 / RPN maps, 96 tiles over 256 slots), with an odd
    # chunk count (the lone last chunk in the last piece of each tile)
    (2, 512, 512, 37, 75), (2, 520, 512, 38, 75),
]


@pytest.mark.parametrize("math", ["bf16x6", "bf16x3"])
@pytest.mark.parametrize("N,Cin,Cout,H,W", SHAPES)
def test_conv_bs_fwd_dgrad(math, N, Cin, Cout, H, W):
    from tlod.conv import conv_dgrad, conv_fwd
    g = torch.Generator().manual_seed(N * 1000 + Cin + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    b = torch.randn(Cout, generator=g)
    y = conv_fwd(x.to(dev), w.to(dev), b.to(dev), relu=False, math=math)
    _close(y, F.conv2d(x.double(), w.double(), b.double(), padding=1), math)
    gy = torch.randn(N, Cout, H, W, generator=g)
    dx = conv_dgrad(gy.to(dev), w.to(dev), math=math)
    _close(dx, torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1), math)


GEMM_SHAPES = [  # N, Cin, Cout, H, W: >= 256 output channels (fwd) / input channels (dgrad)
    (2, 256, 256, 30, 40), (1, 64, 300, 9, 33), (3, 257, 256, 5, 7), (1, 256, 260, 3, 3),
    (1, 300, 512, 16, 16), (2, 512, 256, 37, 75), (1, 128, 256, 1, 40), (1, 16, 256, 40, 2),
]


@pytest.mark.parametrize("math", ["bf16x6", "bf16x3"])
@pytest.mark.parametrize("N,Cin,Cout,H,W", GEMM_SHAPES)
def test_conv_gemm_fwd_dgrad(math, N, Cin, Cout, H, W):
    """tlod_conv3x3_gemm_bs_f32 (im2col rows gathered per 16-deep k chunk, 256x256 tiles,
    split-K slabs on small maps): forward with the full epilogue and dgrad through the
    transposed pack; ragged K = Cin*9, maps narrower than a 4-pixel vector, image 0's first
    rows (the per-dword load path)."""
    from tlod.conv import _conv_gemm, pack_dgrad
    g = torch.Generator().manual_seed(N * 100 + Cin + Cout + H + W)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    b = torch.randn(Cout, generator=g)
    sc = torch.rand(Cout, generator=g) + 0.5
    r = torch.randn(N, Cout, H, W, generator=g)
    y = _conv_gemm(x.to(dev), w.to(dev), 0, b.to(dev), True, sc.to(dev), r.to(dev), Cout, math, "fwd")
    ref = torch.relu(F.conv2d(x.double(), w.double(), padding=1) * sc.double().view(1, -1, 1, 1)
                     + b.double().view(1, -1, 1, 1) + r.double())
    _close(y * (ref > 0).to(dev), ref, math)  # mask flips at f32 rounding of 0 do not count
    y0 = _conv_gemm(x.to(dev), w.to(dev), 0, None, False, None, None, Cout, math, "fwd")
    _close(y0, F.conv2d(x.double(), w.double(), padding=1), math)
    if Cin >= 256:
        gy = torch.randn(N, Cout, H, W, generator=g)
        dx = _conv_gemm(gy.to(dev), pack_dgrad(w.to(dev)), 1, None, False, None, None, Cin, math,
                        "dgrad")
        _close(dx, torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1), math)


def test_conv_gemm_matches_patch_kernel():
    """The implicit-GEMM path and the patch-staged split-bf16 kernel agree to f32 rounding."""
    from tlod.conv import _conv_bs, _conv_gemm, pack_bs
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 256, 40, 60, generator=g).to(dev)
    w = (torch.randn(256, 256, 3, 3, generator=g) * 0.03).to(dev)
    a = _conv_gemm(x, w, 0, None, False, None, None, 256, "bf16x6", "fwd")
    b = _conv_bs(x, pack_bs(w, False), None, False, None, None, 256, 3, "bf16x6", "fwd")
    assert float((a - b).norm() / b.norm()) < 1e-6


WGRAD_SHAPES = SHAPES + [  # + maps narrower than an 8-pixel segment, single rows/columns
    (2, 32, 64, 5, 7), (1, 16, 32, 1, 40), (1, 16, 32, 40, 1), (3, 8, 36, 3, 3),
    (2, 512, 512, 37, 75),
]


@pytest.mark.parametrize("math", ["bf16x6", "bf16x3"])
@pytest.mark.parametrize("N,Cin,Cout,H,W", WGRAD_SHAPES)
def test_conv_bs_wgrad(math, N, Cin, Cout, H, W):
    """tlod_conv_wgrad_bs_f32 (flattened-pixel K, im2col rows staged per chunk) vs fp64,
    plus accumulate=True adding into an existing gradient."""
    from tlod.conv import conv_wgrad
    g = torch.Generator().manual_seed(N * 7 + Cin + Cout + H * 3 + W)
    x = torch.randn(N, Cin, H, W, generator=g)
    gy = torch.randn(N, Cout, H, W, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, 3, 3), gy.double(), padding=1)
    db = torch.empty(Cout, device=dev)
    dw = conv_wgrad(gy.to(dev), x.to(dev), 3, math=math, db=db)
    _close(dw, ref, math)
    # the bias gradient from the same launch (row sums of the staged dy), f32 summation
    _close(db, gy.double().sum((0, 2, 3)), "bf16x6")
    base = torch.randn(Cout, Cin, 3, 3, generator=g)
    acc = base.to(dev).clone()
    conv_wgrad(gy.to(dev), x.to(dev), 3, out=acc, accumulate=True, math=math)
    _close(acc, ref + base.double(), math)


def test_masked_dgrad_is_dgrad_times_mask():
    """tlod_conv_dgrad_bs_mask_f32 = the dgrad with the previous layer's ReLU backward in the
    epilogue: bit-identical to conv_dgrad(...) * (mask > 0), including the split-K tail tiles
    (conv5-shaped map) and the plain-kernel shapes (Cin < 128)."""
    from tlod.conv import conv_dgrad
    g = torch.Generator().manual_seed(3)
    for N, Cin, Cout, H, W in [(2, 512, 512, 37, 75), (1, 64, 128, 40, 57), (2, 256, 256, 75, 150)]:
        gy = torch.randn(N, Cout, H, W, generator=g).to(dev)
        w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).to(dev)
        m = torch.relu(torch.randn(N, Cin, H, W, generator=g)).to(dev)
        a = conv_dgrad(gy, w, math="bf16x6", mask=m)
        b = conv_dgrad(gy, w, math="bf16x6") * (m > 0)
        assert torch.equal(a, b)


def test_fused_relu_backward_chain(monkeypatch):
    """A conv -> conv -> conv chain of fused-ReLU convs: the inner ReLU backward passes run in
    the next conv's dgrad epilogue and the bias gradients come from the wgrad launches
    (STATS counters), with the same gradients as the unfused backward (input gradients
    bit-identical, bias gradients to f32 summation order)."""
    import tlod.conv as tc
    g = torch.Generator().manual_seed(9)
    mods = [tc.Conv2d(c_in, c_out, 3, relu=True).to(dev)
            for c_in, c_out in [(64, 128), (128, 128), (128, 256)]]
    x0 = torch.randn(2, 64, 30, 47, generator=g).to(dev)
    gy = torch.randn(2, 256, 30, 47, generator=g).to(dev)

    def run():
        for m in mods:
            m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = x
        for m in mods:
            y = m(y)
        y.backward(gy)
        return [x.grad] + [t.grad.clone() for m in mods for t in (m.weight, m.bias)]
    before = dict(tc.STATS)
    fused = run()
    assert tc.STATS["masked_dgrad"] - before["masked_dgrad"] == 2
    assert tc.STATS["relu_bwd_skipped"] - before["relu_bwd_skipped"] == 2
    monkeypatch.setattr(tc, "_relu_out", lambda x: False)
    plain = run()
    assert torch.equal(fused[0], plain[0])
    for a, b in zip(fused[1:], plain[1:]):
        _close(a, b.double(), "bf16x6")


def test_conv_bs_wgrad_deterministic_and_f32_accurate():
    """Bitwise repeatable (fixed-order slab sum) and f32-level accurate: normwise error vs
    fp64 within 2.5x of the f32 MFMA wgrad's on a conv3_3-like shape (measured 6.4e-7 vs
    3.6e-7: K = 10800 pixels per output, the 16-deep bf16 MFMA sums add rounding steps)."""
    from tlod.conv import conv_wgrad
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 256, 60, 90, generator=g)
    gy = torch.randn(2, 256, 60, 90, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (256, 256, 3, 3), gy.double(), padding=1)
    a = conv_wgrad(gy.to(dev), x.to(dev), 3, math="bf16x6")
    b = conv_wgrad(gy.to(dev), x.to(dev), 3, math="bf16x6")
    assert torch.equal(a, b)
    f = conv_wgrad(gy.to(dev), x.to(dev), 3, math="f32")

    def err(t):
        return float((t.double().cpu() - ref).norm() / ref.norm())
    assert err(a) <= 2.5 * err(f) + 1e-9, (err(a), err(f))


@pytest.mark.parametrize("math", ["bf16x6"])
def test_conv_bs_epilogue(math):
    from tlod.conv import conv_fwd
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 64, 19, 37, generator=g)
    w = torch.randn(96, 64, 3, 3, generator=g) * 0.05
    sc, sh = torch.rand(96, generator=g) + 0.5, torch.randn(96, generator=g)
    r = torch.randn(2, 96, 19, 37, generator=g)
    y = conv_fwd(x.to(dev), w.to(dev), sh.to(dev), relu=True, scale=sc.to(dev), residual=r.to(dev),
                 math=math)
    ref = F.relu(F.conv2d(x.double(), w.double(), padding=1) * sc.double().view(1, -1, 1, 1)
                 + sh.double().view(1, -1, 1, 1) + r.double())
    _close(y, ref, math)


ONE_SHAPES = [  # N, Cin, Cout, H, W: ResNet101 bottleneck 1x1s (layer2 / layer3 at 600x1200),
    # the 64-, 128- and 256-row tiles, ragged channel / pixel counts
    (2, 1024, 256, 38, 75), (2, 256, 1024, 38, 75), (2, 512, 128, 75, 150), (1, 64, 64, 30, 41),
    (3, 96, 80, 9, 33), (1, 72, 257, 5, 7), (2, 130, 200, 1, 3),
    # the RPN cls / bbox heads on the base feature (18 / 36 outputs: mostly-padding M tiles)
    (2, 512, 18, 37, 75), (2, 512, 36, 37, 75),
]


@pytest.mark.parametrize("math", ["bf16x6", "bf16x3"])
@pytest.mark.parametrize("N,Cin,Cout,H,W", ONE_SHAPES)
def test_conv1x1_gemm_fwd_dgrad(math, N, Cin, Cout, H, W, monkeypatch):
    """1x1 forward (folded-BN scale / shift + residual + ReLU epilogue) and input gradient on
    the split-bf16 conv GEMM (tlod_conv1x1_gemm_bs_f32) vs fp64."""
    from tlod.conv import _gemm1x1, conv_dgrad, conv_fwd
    monkeypatch.setenv("TLOD_CONV1X1_MIN", "16")  # the RPN heads' 18 / 36 outputs
    assert _gemm1x1(1, math, Cin, Cout)
    g = torch.Generator().manual_seed(N * 7 + Cin + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) * (2.0 / Cin) ** 0.5
    sc, sh = torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g)
    r = torch.randn(N, Cout, H, W, generator=g)
    y = conv_fwd(x.to(dev), w.to(dev), sh.to(dev), relu=True, scale=sc.to(dev), residual=r.to(dev),
                 math=math)
    ref = F.relu(F.conv2d(x.double(), w.double()) * sc.double().view(1, -1, 1, 1)
                 + sh.double().view(1, -1, 1, 1) + r.double())
    _close(y, ref, math)
    y0 = conv_fwd(x.to(dev), w.to(dev), None, relu=False, math=math)
    _close(y0, F.conv2d(x.double(), w.double()), math)
    gy = torch.randn(N, Cout, H, W, generator=g)
    dx = conv_dgrad(gy.to(dev), w.to(dev), math=math)
    _close(dx, torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double()), math)


@pytest.mark.parametrize("N,Cin,Cout,H,W", ONE_SHAPES[:4] + ONE_SHAPES[5:6])
def test_conv1x1_dgrad_residual_mask(N, Cin, Cout, H, W):
    """The 1x1 dgrad epilogue with a residual gradient and the previous layer's ReLU mask
    (tlod_conv1x1_gemm_bs_ex_f32): bit-identical to (dgrad + residual) * (mask > 0), including
    split-K tail tiles, and tagged as masked."""
    from tlod.conv import conv_dgrad
    g = torch.Generator().manual_seed(5 + Cin + H)
    gy = torch.randn(N, Cout, H, W, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 1, 1, generator=g) * (2.0 / Cin) ** 0.5).to(dev)
    m = torch.relu(torch.randn(N, Cin, H, W, generator=g)).to(dev)
    r = torch.randn(N, Cin, H, W, generator=g).to(dev)
    a = conv_dgrad(gy, w, math="bf16x6", mask=m, residual=r)
    b = (conv_dgrad(gy, w, math="bf16x6") + r) * (m > 0)
    assert torch.equal(a, b)
    assert a._tlod_relu_masked[0] == m.data_ptr()
    c = conv_dgrad(gy, w, math="bf16x6", mask=m)
    assert torch.equal(c, conv_dgrad(gy, w, math="bf16x6") * (m > 0))


def test_bottleneck_shortcut_link_matches_unfused(monkeypatch):
    """Two identity ResNet bottlenecks (layer3-like widths): with the ShortcutLink the
    shortcut gradient is added in conv1's dgrad epilogue before the previous block's ReLU
    mask, and the masked gradient skips that block's ReLU-backward pass; input and weight
    gradients equal the unlinked backward's (the same kernels, summed in the same order)."""
    import tlod.conv as tc
    from tlod.detector import resnet as rn
    torch.manual_seed(4)
    blocks = torch.nn.Sequential(rn.Bottleneck(512, 128), rn.Bottleneck(512, 128)).to(dev)
    for m in blocks.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eval()
            m.weight.requires_grad_(False)
            m.bias.requires_grad_(False)
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    x0 = torch.relu(torch.randn(2, 512, 19, 38)).to(dev)
    gy = torch.randn(2, 512, 19, 38).to(dev)

    def run():
        blocks.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = tc.ConvBNFunction.apply(x, torch.ones(512, 512, 1, 1, device=dev) * 0.01,
                                    torch.ones(512, device=dev), torch.zeros(512, device=dev),
                                    None, True, None, 0)  # a ReLU output feeding block 0
        blocks(y).backward(gy)
        return [x.grad] + [p.grad.clone() for p in blocks.parameters() if p.requires_grad]
    before = dict(tc.STATS)
    linked = run()
    n_skip = tc.STATS["relu_bwd_skipped"] - before["relu_bwd_skipped"]
    monkeypatch.setattr(rn, "ShortcutLink", lambda: None)
    before = dict(tc.STATS)
    plain = run()
    assert n_skip > tc.STATS["relu_bwd_skipped"] - before["relu_bwd_skipped"]
    for a, b in zip(linked, plain):
        _close(a, b.double(), "bf16x6")


def test_conv_bs_matches_f32_path_closely():
    """bf16x6 and the f32-input MFMA path agree to f32 rounding on a conv3_3 shape."""
    from tlod.conv import conv_fwd
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 256, 75, 125, generator=g).to(dev)
    w = (torch.randn(256, 256, 3, 3, generator=g) * 0.03).to(dev)
    a = conv_fwd(x, w, None, False, math="f32")
    b = conv_fwd(x, w, None, False, math="bf16x6")
    assert float((a - b).norm() / a.norm()) < 1e-6


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 256, 256, 30, 40), (1, 64, 128, 75, 150)])
def test_bf16x6_as_accurate_as_f32_mfma(N, Cin, Cout, H, W):
    """The default split-bf16 math is no less accurate than the f32-input MFMA path: its
    normwise error vs fp64 is within 1.5x of the f32 path's on the same data."""
    from tlod.conv import conv_dgrad, conv_fwd
    g = torch.Generator().manual_seed(Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    gy = torch.randn(N, Cout, H, W, generator=g)
    ref_y = F.conv2d(x.double(), w.double(), padding=1)
    ref_dx = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1)

    def err(a, r):
        return float((a.detach().double().cpu() - r).norm() / r.norm())
    e = {m: (err(conv_fwd(x.to(dev), w.to(dev), None, False, math=m), ref_y),
             err(conv_dgrad(gy.to(dev), w.to(dev), math=m), ref_dx)) for m in ("f32", "bf16x6")}
    assert e["bf16x6"][0] <= 1.5 * e["f32"][0] + 1e-9, e
    assert e["bf16x6"][1] <= 1.5 * e["f32"][1] + 1e-9, e


def test_split_bf16_huge_finite_operands():
    """Finite operands whose round-to-nearest bf16 hi would be infinite (|x| >= 0x7f7f8000,
    ~3.396e38) keep the truncated hi: conv fwd / dgrad / wgrad and the GEMM give
    finite results at f32-level error instead of NaN."""
    from tlod.conv import conv_dgrad, conv_fwd, conv_wgrad
    from tlod.linear import gemm
    big = 3.4e38
    assert big > 3.3961e38 and big < torch.finfo(torch.float32).max
    g = torch.Generator().manual_seed(21)
    x = torch.randn(1, 16, 12, 20, generator=g)
    x[0, 3, 4, 5], x[0, 9, 10, 17], x[0, 15, 0, 0] = big, -big, big
    w = torch.randn(32, 16, 3, 3, generator=g) * 1e-3
    y = conv_fwd(x.to(dev), w.to(dev), None, False, math="bf16x6")
    assert torch.isfinite(y).all()
    _close(y, F.conv2d(x.double(), w.double(), padding=1), "bf16x6")
    gy = torch.randn(1, 32, 12, 20, generator=g)
    wb = w.clone()
    wb[5, 3, 1, 1] = -big
    dx = conv_dgrad(gy.to(dev) * 1e-3, wb.to(dev), math="bf16x6")
    assert torch.isfinite(dx).all()
    _close(dx, torch.nn.grad.conv2d_input(x.shape, wb.double(), gy.double() * 1e-3, padding=1),
           "bf16x6")
    dw = conv_wgrad(gy.to(dev) * 1e-3, x.to(dev), 3, math="bf16x6")
    assert torch.isfinite(dw).all()
    _close(dw, torch.nn.grad.conv2d_weight(x.double(), (32, 16, 3, 3), gy.double() * 1e-3,
                                           padding=1), "bf16x6")
    A = torch.randn(40, 64, generator=g)
    A[3, 7], A[20, 63] = big, -big
    B = torch.randn(24, 64, generator=g) * 1e-3
    c = gemm(A.to(dev), B.to(dev), 40, 24, 64, 1, 1, None, "bf16x6")
    assert torch.isfinite(c).all()
    _close(c, A.double() @ B.double().t(), "bf16x6")


def test_fused_relu_backward_multi_consumer(monkeypatch):
    """A fused-ReLU conv output read by two consumers (the next conv and a side branch): the
    next conv's masked dgrad is summed with the branch's gradient by autograd (possibly in
    place into the tagged tensor), so the ReLU backward must NOT be skipped; the gradients
    equal the unfused backward's."""
    import tlod.conv as tc
    g = torch.Generator().manual_seed(12)
    c1, c2 = tc.Conv2d(32, 64, 3, relu=True).to(dev), tc.Conv2d(64, 64, 3, relu=True).to(dev)
    x0 = torch.randn(1, 32, 20, 28, generator=g).to(dev)
    gy = torch.randn(1, 64, 20, 28, generator=g).to(dev)
    side = torch.randn(1, 64, 20, 28, generator=g).to(dev)

    def run():
        for m in (c1, c2):
            m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y1 = c1(x)
        loss = (c2(y1) * gy).sum() + (y1 * side).sum()
        loss.backward()
        return [x.grad, c1.weight.grad.clone(), c1.bias.grad.clone(), c2.weight.grad.clone()]
    before = dict(tc.STATS)
    fused = run()
    assert tc.STATS["masked_dgrad"] - before["masked_dgrad"] == 1
    assert tc.STATS["relu_bwd_skipped"] == before["relu_bwd_skipped"]
    monkeypatch.setattr(tc, "_relu_out", lambda x: False)
    plain = run()
    for a, b in zip(fused, plain):
        _close(a, b.double(), "bf16x6")


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 3, 64, 600, 1200), (1, 3, 64, 37, 300), (1, 1, 7, 5, 260),
                                           (3, 4, 20, 9, 8)])
def test_conv3x3_direct(N, Cin, Cout, H, W):
    """Direct f32 3x3 conv for Cin <= 4 (VGG16 conv1_1 on the image, fused bias + ReLU) vs
    fp64: f32 FMA chains, 1e-6 normwise."""
    from tlod.conv import conv_fwd
    g = torch.Generator().manual_seed(Cin * 100 + Cout + W)
    x = torch.randn(N, Cin, H, W, generator=g) * 50
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.2
    b = torch.randn(Cout, generator=g)
    for relu in (True, False):
        y = conv_fwd(x.to(dev), w.to(dev), b.to(dev), relu=relu)
        ref = F.conv2d(x.double(), w.double(), b.double(), padding=1)
        ref = F.relu(ref) if relu else ref
        got = y.double().cpu()
        assert float((got - ref).norm() / ref.norm()) < 1e-6


def _ref_pack(w, dgrad):
    """The packed split-bf16 planes of tlod_conv_pack_bs (conv.hip pack_bs_kernel) built with
    torch ops: rows x chunks x 10 tap slots x 8 channels per plane, dgrad = the transposed,
    tap-flipped operand; hi = the truncated bf16 of w, mid / lo the round-to-nearest-even
    bf16 of the remainders (bs_common.h split2)."""
    Cout, Cin = w.shape[:2]
    a = w.permute(1, 0, 2, 3).flip(2, 3) if dgrad else w
    rows, ins = a.shape[:2]
    nch = (ins + 7) // 8
    A = torch.zeros(rows, nch * 8, 10, dtype=torch.float32)
    A[:, :ins, :9] = a.reshape(rows, ins, 9)
    A = A.view(rows, nch, 8, 10).permute(0, 1, 3, 2).contiguous().view(-1)
    u = A.view(torch.int32)
    hi = (u & -65536).view(torch.float32)
    r = A - hi
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return torch.cat([(u >> 16).to(torch.int16), mid.view(torch.int16), lo.view(torch.int16)])


@pytest.mark.parametrize("Cout,Cin", [(64, 3), (64, 64), (128, 64), (512, 512), (20, 13),
                                      (132, 130), (33, 517)])
@pytest.mark.parametrize("dgrad", [False, True])
def test_pack_bs_bit_exact(Cout, Cin, dgrad):
    """tlod_conv_pack_bs bit-exact vs the torch construction, including ragged channel
    counts (Cin / Cout not a multiple of 8) and the dgrad transpose + tap flip."""
    from tlod.conv import _pack_bs
    g = torch.Generator().manual_seed(Cout * 1000 + Cin)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * torch.exp(torch.randn(Cout, Cin, 3, 3, generator=g))
    p = _pack_bs(w.to(dev), dgrad).view(torch.int16).cpu()
    ref = _ref_pack(w, dgrad)
    assert p.numel() == ref.numel()
    assert torch.equal(p, ref)



@pytest.mark.parametrize("KS,N,Cin,Cout,H,W", [(1, 2, 256, 1024, 19, 38), (1, 2, 1024, 256, 19, 38),
                                              (3, 2, 256, 256, 19, 38), (3, 1, 64, 72, 30, 41)])
def test_bn_scale_folded_into_dgrad_and_wgrad(KS, N, Cin, Cout, H, W):
    """A frozen BatchNorm's per-channel scale after the conv, folded into the dgrad (staged
    weight for 1x1, tlod_conv_pack_bs_ex for 3x3) and the wgrad reduce
    (tlod_conv_wgrad_bs_ex_f32): bit-identical to scaling the weight / the weight gradient
    with a separate pass (ConvBNFunction's skipped-ReLU path, round 4)."""
    from tlod.conv import conv_dgrad, conv_wgrad
    g = torch.Generator().manual_seed(KS * 100 + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, KS, KS, generator=g) * (2.0 / (Cin * KS * KS)) ** 0.5).to(dev)
    s = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    gy = torch.randn(N, Cout, H, W, generator=g).to(dev)
    m = torch.relu(torch.randn(N, Cin, H, W, generator=g)).to(dev)
    a = conv_dgrad(gy, w, math="bf16x6", mask=m, wscale=s)
    b = conv_dgrad(gy, w * s.view(-1, 1, 1, 1), math="bf16x6", mask=m)
    assert torch.equal(a, b)
    dw = conv_wgrad(gy, x, KS, math="bf16x6", row_scale=s)
    assert torch.equal(dw, conv_wgrad(gy, x, KS, math="bf16x6") * s.view(-1, 1, 1, 1))


@pytest.mark.parametrize("KS,N,Cin,Cout,H,W", [(1, 2, 256, 1024, 19, 38), (3, 2, 256, 256, 19, 38),
                                              (3, 1, 64, 72, 30, 41),
                                              # row length Cin * KS * KS = 18 (KS = 1) / 18
                                              # (KS = 3): float4s of the slab reduce straddle rows
                                              (1, 1, 18, 2, 9, 13), (3, 1, 2, 2, 9, 13)])
def test_wgrad_row_scale_accumulate(KS, N, Cin, Cout, H, W):
    """tlod_conv_wgrad_bs_ex_f32 with accumulate=True and a row scale: out = base + s * dW
    (the reduce's dW + r * sum), on the 1x1 im2col path, the 3x3 wgrad_ws path, and row
    lengths that are not a multiple of 4 (round-4 advisor: the scale was taken per float4)."""
    from tlod.conv import conv_wgrad
    g = torch.Generator().manual_seed(KS * 1000 + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g).to(dev)
    gy = torch.randn(N, Cout, H, W, generator=g).to(dev)
    s = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    base = torch.randn(Cout, Cin, KS, KS, generator=g).to(dev)
    dw = conv_wgrad(gy, x, KS, math="bf16x6")
    got = conv_wgrad(gy, x, KS, out=base.clone(), accumulate=True, math="bf16x6", row_scale=s)
    torch.testing.assert_close(got, base + dw * s.view(-1, 1, 1, 1), rtol=1e-6, atol=1e-6)
    scaled = conv_wgrad(gy, x, KS, math="bf16x6", row_scale=s)
    assert torch.equal(scaled, dw * s.view(-1, 1, 1, 1))
