"""1x1 convolutions with 1..4 output channels (tlod_conv1x1_small_*: _ImageDA.Conv2, 512 -> 2,
lib/DAF/DA.py:36-50) vs a PyTorch fp64 reference: forward, input gradient, weight and bias
gradients, on both the float4 (H*W % 4 == 0) and scalar paths, and bit-identical repeats.
Bars as the f32 conv tests: normwise relative 1e-5, elementwise 1e-4 of max|ref|."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _close(got, ref, tol=1e-5, etol=1e-4):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    nrm = float((got - ref).norm() / max(float(ref.norm()), 1e-30))
    assert nrm <= tol, f"normwise rel err {nrm:.3e}"
    assert float((got - ref).abs().max()) <= etol * float(ref.abs().max()) + 1e-30


@pytest.mark.parametrize("N,Cin,H,W,Cout,bias", [
    (2, 512, 37, 75, 2, False),    # DAF-VGG16 conv5_3 map (H*W odd: scalar path)
    (2, 256, 150, 300, 2, False),  # ATF-R101 layer1 map (float4 path)
    (1, 1024, 38, 75, 2, False),   # layer3 map (H*W % 4 == 2)
    (2, 64, 8, 12, 3, True),
    (1, 7, 5, 5, 1, True),
    (3, 33, 16, 16, 4, True),
])
def test_conv1x1_small_matches_fp64(N, Cin, H, W, Cout, bias):
    from tlod.conv import Conv1x1SmallFunction
    g = torch.Generator().manual_seed(N * 1000 + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) * 0.05
    b = torch.randn(Cout, generator=g) if bias else None
    dy = torch.randn(N, Cout, H, W, generator=g)
    xd = x.double().requires_grad_()
    wd = w.double().requires_grad_()
    bd = b.double().requires_grad_() if bias else None
    yr = F.conv2d(xd, wd, bd)
    yr.backward(dy.double())
    xg = x.to(dev).requires_grad_()
    wg = w.to(dev).requires_grad_()
    bg = b.to(dev).requires_grad_() if bias else None
    y = Conv1x1SmallFunction.apply(xg, wg, bg)
    y.backward(dy.to(dev))
    _close(y, yr)
    _close(xg.grad, xd.grad)
    _close(wg.grad, wd.grad)
    if bias:
        _close(bg.grad, bd.grad)
    # deterministic: the same bits again
    xg2 = x.to(dev).requires_grad_()
    wg2 = w.to(dev).requires_grad_()
    y2 = Conv1x1SmallFunction.apply(xg2, wg2, bg)
    y2.backward(dy.to(dev))
    assert torch.equal(y, y2) and torch.equal(xg.grad, xg2.grad) and torch.equal(wg.grad, wg2.grad)


def test_imageda_head_uses_small_conv():
    """_ImageDA.Conv2 (512 -> 2, no bias) dispatches to the streaming kernels and matches the
    nn.Conv2d arithmetic of the reference module (fp64)."""
    from tlod.conv import Conv2d
    torch.manual_seed(3)
    m = Conv2d(512, 2, 1, bias=False).to(dev)
    x = torch.randn(2, 512, 37, 75, device=dev, requires_grad=True)
    y = m(x)
    assert type(y.grad_fn).__name__.startswith("Conv1x1SmallFunction")
    y.sum().backward()
    xd = x.detach().double().cpu().requires_grad_()
    wd = m.weight.detach().double().cpu().requires_grad_()
    yr = F.conv2d(xd, wd)
    yr.sum().backward()
    _close(y, yr)
    _close(x.grad, xd.grad)
    _close(m.weight.grad, wd.grad)
