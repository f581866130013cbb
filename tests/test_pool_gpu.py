"""2x2 max pooling (nn.MaxPool2d(2, 2), floor mode) in libtlod vs torch: forward values,
the fused argmax-routing + ReLU backward (bit-exact against torch's max_pool2d / relu
autograd, ties and odd sizes included), the conv epilogue pooling of frozen layers, and
the conv + ReLU + pool autograd node (vs fp64)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.mark.parametrize("N,C,H,W", [(2, 3, 8, 10), (1, 5, 7, 9), (2, 64, 150, 300), (1, 2, 2, 2),
                                     (1, 4, 3, 33)])
def test_maxpool_fwd_bwd_exact(N, C, H, W):
    from tlod.conv import maxpool2x2, maxpool_relu_bwd
    g = torch.Generator().manual_seed(N + C + H + W)
    z = torch.randn(N, C, H, W, generator=g)
    z[z.abs() < 0.3] = 0.0           # ReLU zeros: all-zero windows and ties
    if H > 1:  # exact ties between the two rows of some windows
        z[:, :, 0::2][:, :, :, ::3] = z[:, :, 1::2][:, :, :z[:, :, 0::2].shape[2]][:, :, :, ::3] \
            if z.shape[2] % 2 == 0 else z[:, :, 0::2][:, :, :, ::3]
    zd = z.to(dev).requires_grad_(True)
    y = F.relu(zd)
    p = F.max_pool2d(y, 2, 2)
    dp = torch.randn(p.shape, generator=g).to(dev)
    p.backward(dp)
    got = maxpool2x2(y.detach())
    assert torch.equal(got, p.detach())
    gg, db = maxpool_relu_bwd(dp, y.detach())
    assert torch.equal(gg, zd.grad)
    # db: a different summation order than torch's reduction; bound by the sum of |g|
    ref = zd.grad.double().sum((0, 2, 3))
    bound = 1e-6 * zd.grad.double().abs().sum((0, 2, 3)) + 1e-7
    assert bool(((db.double() - ref).abs() <= bound).all())


def test_maxpool_nan_propagates_like_torch():
    from tlod.conv import maxpool2x2
    x = torch.tensor([[[[1.0, float("nan"), 3.0, 4.0], [0.0, 2.0, 5.0, 1.0]]]], device=dev)
    got, ref = maxpool2x2(x), F.max_pool2d(x, 2, 2)
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(got[~torch.isnan(got)], ref[~torch.isnan(ref)])


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 3, 64, 40, 70), (2, 64, 64, 37, 75),
                                            (1, 64, 128, 33, 31), (1, 128, 128, 32, 64)])
def test_conv_epilogue_pool(N, Cin, Cout, H, W):
    """Frozen conv + ReLU + pool with the pooling in the split-bf16 conv epilogue."""
    from tlod.conv import conv_fwd_pool
    g = torch.Generator().manual_seed(Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    got = conv_fwd_pool(x.to(dev), w.to(dev), b.to(dev))
    ref = F.max_pool2d(F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1)), 2, 2)
    err = float((got.double().cpu() - ref).norm() / ref.norm())
    assert got.shape == ref.shape and err < 1e-5, err


def test_conv_pool_module_grads():
    """Conv2d(pool=True) with trainable weights: conv -> ReLU -> pool autograd node."""
    from tlod.conv import Conv2d
    torch.manual_seed(3)
    m = Conv2d(32, 64, 3, relu=True)
    m.pool = True
    ref = torch.nn.Conv2d(32, 64, 3, padding=1).double()
    ref.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
    m = m.to(dev)
    x = torch.randn(2, 32, 19, 30)
    xd = x.to(dev).requires_grad_(True)
    y = m(xd)
    xr = x.double().requires_grad_(True)
    yr = F.max_pool2d(F.relu(ref(xr)), 2, 2)
    dy = torch.randn(yr.shape)
    y.backward(dy.to(dev))
    yr.backward(dy.double())
    for a, b in ((y, yr), (xd.grad, xr.grad), (m.weight.grad, ref.weight.grad),
                 (m.bias.grad, ref.bias.grad)):
        e = float((a.detach().double().cpu() - b).norm() / b.norm())
        assert e < 1e-5, e
