"""HIP implicit-GEMM convolution (f32 MFMA) vs a plain PyTorch fp64 CPU reference.

Bar (north star: 1e-3 relative for conv activations): we require normwise relative
error <= 1e-5 and elementwise |err| <= 1e-4 * max|ref| — the f32-input MFMA computes an
exact f32 FMA chain, so the error is f32 rounding only.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _close(got, ref, tol=1e-5):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    nrm = (got - ref).norm() / max(ref.norm(), 1e-30)
    assert nrm <= tol, f"normwise rel err {nrm:.3e}"
    assert (got - ref).abs().max() <= 1e-4 * ref.abs().max() + 1e-30


SHAPES = [  # N, Cin, Cout, H, W, KS
    (2, 64, 128, 37, 75, 3), (1, 3, 64, 50, 70, 3), (2, 256, 256, 30, 40, 3),
    (1, 512, 512, 37, 62, 3), (1, 32, 64, 5, 7, 3), (1, 130, 132, 9, 33, 3),
    (2, 512, 512, 20, 31, 1), (1, 512, 24, 37, 62, 1), (1, 512, 48, 11, 13, 1),
]


@pytest.mark.parametrize("math", ["f32", "bf16x6"])
@pytest.mark.parametrize("N,Cin,Cout,H,W,KS", SHAPES)
def test_conv_fwd_bwd(N, Cin, Cout, H, W, KS, math, monkeypatch):
    monkeypatch.setenv("TLOD_CONV_MATH", math)
    from tlod.conv import ConvFunction
    g = torch.Generator().manual_seed(N * 1000 + Cin + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, KS, KS, generator=g) * (2.0 / (Cin * KS * KS)) ** 0.5
    b = torch.randn(Cout, generator=g)
    for relu in (False, True):
        xd, wd, bd = (t.to(dev).requires_grad_(True) for t in (x, w, b))
        y = ConvFunction.apply(xd, wd, bd, relu)
        xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
        yr = F.conv2d(xr, wr, br, padding=KS // 2)
        if relu:
            _close(y, F.relu(yr))
            # backward through the device's ReLU mask: a pre-activation within f32
            # rounding of 0 may flip the mask between fp32 and fp64 (seen: 1 of 1.2M)
            yr = yr * (y.detach().cpu() > 0).double()
        _close(y, yr)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy.to(dev))
        yr.backward(gy.double())
        _close(xd.grad, xr.grad)
        _close(wd.grad, wr.grad)
        _close(bd.grad, br.grad)


def test_conv_module_matches_nn_conv2d_keys():
    from tlod.conv import Conv2d
    m = Conv2d(64, 128, 3, relu=True)
    ref = torch.nn.Conv2d(64, 128, 3, padding=1)
    assert m.state_dict().keys() == ref.state_dict().keys()
    assert m.weight.shape == ref.weight.shape


def test_wgrad_deterministic():
    from tlod.conv import conv_wgrad
    g = torch.randn(2, 256, 40, 60, device=dev)
    x = torch.randn(2, 128, 40, 60, device=dev)
    a = conv_wgrad(g, x, 3)
    b = conv_wgrad(g, x, 3)
    assert torch.equal(a, b)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 512, 512, 37, 75), (1, 512, 512, 12, 20),
                                            (2, 256, 512, 38, 40), (1, 64, 256, 150, 250)])
@pytest.mark.parametrize("math", ["f32", "bf16x6"])
def test_conv_split_k_paths(N, Cin, Cout, H, W, math, monkeypatch):
    monkeypatch.setenv("TLOD_CONV_MATH", math)
    _split_k_case(N, Cin, Cout, H, W)


def _split_k_case(N, Cin, Cout, H, W):
    """Small maps split every tile over input channels; larger ones (the last shape: 608
    tiles on 512 slots) split only the tail round.  Both go through the slab + reduce."""
    from tlod import _lib
    from tlod.conv import conv_dgrad, conv_fwd
    assert _lib.lib().tlod_conv_fwd_workspace_bytes(N, Cin, H, W, Cout, 3) > 0
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    b = torch.randn(Cout, generator=g)
    y = conv_fwd(x.to(dev), w.to(dev), b.to(dev), relu=True)
    _close(y, F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1)))
    gy = torch.randn(N, Cout, H, W, generator=g)
    dx = conv_dgrad(gy.to(dev), w.to(dev))
    _close(dx, torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1))
    y2 = conv_fwd(x.to(dev), w.to(dev), b.to(dev), relu=True)
    assert torch.equal(y, y2)  # deterministic
