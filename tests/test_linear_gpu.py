"""Split-bf16 GEMM (tlod_gemm_bs_f32) and tlod.linear.Linear vs a PyTorch fp64 CPU
reference.

Bars (normwise relative / elementwise vs max|ref|): bf16x6 1e-5 / 1e-4 — f32-level error
(the three bf16 planes carry the f32 mantissa exactly, the dropped cross terms are below
2^-24 relative); bf16x3 5e-5 / 5e-4.  Every operand layout (K- or M/N-contiguous), ragged
M/N/K (tile edges, K tails inside a 16-deep chunk, odd strides for the unaligned loads),
the split-K path and the head's real shapes (fc6 / fc7 with 556 RoIs).
"""
import pytest
import torch

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


@pytest.mark.parametrize("math", ["bf16x6", "bf16x3"])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K", [(556, 300, 1000), (1, 7, 3), (37, 513, 17), (256, 256, 16),
                                   (300, 1024, 4105), (5, 3000, 64)])
def test_gemm_layouts(M, N, K, ak, bk, math):
    from tlod.linear import gemm
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + 10 * ak + bk)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    a = A if ak else A.t().contiguous()
    b = B if bk else B.t().contiguous()
    c = gemm(a.to(dev), b.to(dev), M, N, K, ak, bk, bias.to(dev), math)
    _close(c, A.double() @ B.double().t() + bias.double(), math)


def test_gemm_split_k_deterministic():
    """A deep-K / few-tile product takes the split-K slab path; results repeat bitwise."""
    from tlod import _lib
    from tlod.linear import gemm
    M, N, K = 300, 512, 25088
    assert _lib.lib().tlod_gemm_bs_workspace_bytes(M, N, K, 1, 1, 6) > 0
    g = torch.Generator().manual_seed(1)
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    c1 = gemm(A.to(dev), B.to(dev), M, N, K, 1, 1)
    c2 = gemm(A.to(dev), B.to(dev), M, N, K, 1, 1)
    assert torch.equal(c1, c2)
    _close(c1, A.double() @ B.double().t(), "bf16x6")


@pytest.mark.parametrize("R,I,O", [(556, 25088, 4096), (556, 4096, 4096), (556, 4096, 1024),
                                   (256, 4096, 9), (256, 4096, 36), (556, 1024, 1), (556, 2048, 9),
                                   (256, 4105, 1024), (3, 100, 20)])
def test_linear_fwd_bwd(R, I, O):
    """tlod.linear.Linear forward, input / weight / bias gradients vs nn.Linear in fp64."""
    from tlod.linear import Linear
    torch.manual_seed(R + I + O)
    lin = Linear(I, O)
    ref = torch.nn.Linear(I, O).double()
    ref.load_state_dict({k: v.double() for k, v in lin.state_dict().items()})
    lin = lin.to(dev)
    x = torch.randn(R, I)
    gy = torch.randn(R, O)
    xd = x.to(dev).requires_grad_(True)
    y = lin(xd)
    y.backward(gy.to(dev))
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy.double())
    _close(y, yr, "bf16x6")
    _close(xd.grad, xr.grad, "bf16x6")
    _close(lin.weight.grad, ref.weight.grad, "bf16x6")
    _close(lin.bias.grad, ref.bias.grad, "bf16x6")


def test_linear_state_dict_matches_nn_linear():
    from tlod.linear import Linear
    a, b = Linear(25088, 4096), torch.nn.Linear(25088, 4096)
    assert a.state_dict().keys() == b.state_dict().keys()
    assert a.weight.shape == b.weight.shape and a.bias.shape == b.bias.shape


def test_relu_dropout_fused():
    """tlod_relu_dropout_f32: p = 0 is exactly ReLU; at p = 0.5 about half the positive
    entries survive, scaled by 2; the backward routes dout through exactly the surviving
    entries (x2) — the same function torch's relu + dropout computes for that mask."""
    from tlod.linear import ReluDropoutFunction
    g = torch.Generator().manual_seed(0)
    y = torch.randn(556, 4096, generator=g).to(dev)
    out0 = ReluDropoutFunction.apply(y, 0.0, 123)
    assert torch.equal(out0, torch.relu(y))
    yr = y.clone().requires_grad_(True)
    out = ReluDropoutFunction.apply(yr, 0.5, 123)
    pos = y > 0
    kept = out > 0
    assert not bool((kept & ~pos).any())
    frac = float(kept.sum()) / float(pos.sum())
    assert abs(frac - 0.5) < 0.01, frac
    assert torch.equal(out[kept], y[kept] * 2.0)
    dout = torch.randn(y.shape, generator=g).to(dev)
    out.backward(dout)
    assert torch.equal(yr.grad, torch.where(kept, dout * 2.0, torch.zeros_like(dout)))
    # same seed, same mask; another seed, another mask
    assert torch.equal(ReluDropoutFunction.apply(y, 0.5, 123), out.detach())
    assert not torch.equal(ReluDropoutFunction.apply(y, 0.5, 124), out.detach())


def test_relu_dropout_passes_nan_like_torch():
    """NaN must reach the loss as NaN (torch.relu / nn.Dropout propagate it), and
    the backward passes the gradient at a NaN output as torch's threshold_backward does."""
    from tlod.linear import ReluDropoutFunction
    y = torch.tensor([1.0, -1.0, float("nan"), 0.0, 2.0, float("nan"), -3.0, 4.0], device=dev)
    yr = y.clone().requires_grad_(True)
    out = ReluDropoutFunction.apply(yr, 0.0, 0)
    ref = torch.relu(y)
    assert torch.equal(torch.isnan(out), torch.isnan(ref))
    ok = ~torch.isnan(ref)
    assert torch.equal(out[ok], ref[ok])
    dout = torch.arange(1.0, 9.0, device=dev)
    out.backward(dout)
    yt = y.clone().requires_grad_(True)
    torch.relu(yt).backward(dout)
    assert torch.equal(yr.grad, yt.grad)


def test_relu_dropout_p0_leaves_cpu_rng_alone():
    """no seed draw from torch's CPU generator when dropout is off."""
    from tlod.linear import relu_dropout
    d = torch.nn.Dropout(0.5).eval()
    torch.manual_seed(5)
    a = torch.rand(3)
    torch.manual_seed(5)
    relu_dropout(torch.randn(64, device=dev), d)
    b = torch.rand(3)
    assert torch.equal(a, b)


@pytest.mark.parametrize("R,H,W,C,O", [(1, 4, 4, 256, 256), (37, 4, 4, 512, 512), (300, 4, 4, 256, 512),
                                       (3, 5, 7, 256, 48), (2, 1, 3, 512, 16)])
def test_gemm_nhwc3_modes(R, H, W, C, O):
    """tlod_gemm_nhwc3_bs_f32: the RoI head's 3x3 conv as implicit GEMMs over channels-last
    maps vs torch fp64 — forward with the bias / residual / ReLU epilogue, the input gradient
    with the residual + ReLU-mask epilogue (through the tap-flipped weight), the weight
    gradient; ragged map sizes (5 x 7, 1 x 3: every tap border), split-K tails (R = 1)."""
    import torch.nn.functional as F
    from tlod.linear import gemm_nhwc3
    g = torch.Generator().manual_seed(R * 31 + C + O + W)
    x = torch.randn(R, H, W, C, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5
    dy = torch.randn(R, H, W, O, generator=g)
    bias, res = torch.randn(O, generator=g), torch.randn(R, H, W, O, generator=g)
    xc = x.permute(0, 3, 1, 2).double()
    wm = w.permute(0, 2, 3, 1).reshape(O, 9 * C)
    rows = R * H * W
    # forward (plain and with the full epilogue)
    ref = F.conv2d(xc, w.double(), padding=1).permute(0, 2, 3, 1).reshape(rows, O)
    y = gemm_nhwc3(0, x.reshape(rows, C).to(dev), wm.to(dev), R, H, W, C, O)
    _close(y, ref, "bf16x6")
    y = gemm_nhwc3(0, x.reshape(rows, C).to(dev), wm.to(dev), R, H, W, C, O, bias=bias.to(dev),
                   residual=res.reshape(rows, O).to(dev), relu=True)
    refe = torch.relu(ref + bias.double() + res.reshape(rows, O).double())
    _close(y * (refe > 0).to(dev), refe, "bf16x6")  # (mask flips at f32 rounding of 0)
    # input gradient
    wd = wm.view(O, 9, C).flip(1).transpose(0, 1).reshape(9 * O, C)
    refd = torch.nn.grad.conv2d_input(xc.shape, w.double(), dy.permute(0, 3, 1, 2).double(),
                                      padding=1).permute(0, 2, 3, 1).reshape(rows, C)
    dx = gemm_nhwc3(1, dy.reshape(rows, O).to(dev), wd.to(dev), R, H, W, C, O)
    _close(dx, refd, "bf16x6")
    m = torch.relu(torch.randn(rows, C, generator=g))
    r2 = torch.randn(rows, C, generator=g)
    dxm = gemm_nhwc3(1, dy.reshape(rows, O).to(dev), wd.to(dev), R, H, W, C, O,
                     residual=r2.to(dev), mask=m.to(dev))
    assert torch.equal(dxm, (dx + r2.to(dev)) * (m.to(dev) > 0))
    # weight gradient, in the (O, 9C) GEMM layout
    refw = torch.nn.grad.conv2d_weight(xc, (O, C, 3, 3), dy.permute(0, 3, 1, 2).double(),
                                       padding=1).permute(0, 2, 3, 1).reshape(O, 9 * C)
    dw = gemm_nhwc3(2, dy.reshape(rows, O).to(dev), x.reshape(rows, C).to(dev), R, H, W, C, O)
    _close(dw, refw, "bf16x6")
