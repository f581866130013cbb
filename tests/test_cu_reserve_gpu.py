"""The kernels' round planners under a CU reserve (tlod_set_cu_reserve, runtime.hip
cached_slots): while the data-parallel all-reduces run, tlod.dist.GradBucketReducer plans
every split-K / tail round for (CUs - reserve) slots, so the 8-GPU run executes plans that a
1-GPU run never does (the reference's DataParallel path this replaces is
methods/DAF/DAF_train.py:341-342).  Here the conv fwd / dgrad (warp-specialized and plain),
the 3x3 weight gradient (wgrad_ws), the 1x1 conv GEMMs and the head GEMM run under a reserve
of 32 CUs (the nccl default) and of 37 (an odd count: no shape's plan is a power of two), with
the workspace queried and the launch made under that same reserve, against fp64 at the
ordinary bars — and the reserve really re-plans (the split-K workspaces change).
"""
import pytest
import torch
import torch.nn.functional as F

import test_conv_bs_gpu as tcb
import test_linear_gpu as tlg

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(params=[32, 37])
def reserve(request):
    from tlod import _lib
    L = _lib.lib()
    _lib.check(L.tlod_set_cu_reserve(request.param), "set_cu_reserve")
    yield request.param
    _lib.check(L.tlod_set_cu_reserve(0), "set_cu_reserve")


CONV_SHAPES = [  # ws kernel (conv3_3 map), conv5 / RPN map (split-K tails), plain Cin = 64,
    # ragged channels
    (2, 256, 256, 150, 250), (2, 512, 512, 37, 75), (1, 64, 256, 150, 250), (1, 130, 132, 9, 33),
    (1, 128, 136, 75, 150)]


@pytest.mark.parametrize("N,Cin,Cout,H,W", CONV_SHAPES)
def test_conv_fwd_dgrad_under_reserve(reserve, N, Cin, Cout, H, W):
    tcb.test_conv_bs_fwd_dgrad("bf16x6", N, Cin, Cout, H, W)


@pytest.mark.parametrize("N,Cin,Cout,H,W", CONV_SHAPES + [(2, 512, 512, 37, 75), (3, 8, 36, 3, 3)])
def test_conv_wgrad_under_reserve(reserve, N, Cin, Cout, H, W):
    tcb.test_conv_bs_wgrad("bf16x6", N, Cin, Cout, H, W)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 1024, 256, 38, 75), (2, 256, 1024, 38, 75),
                                           (2, 512, 128, 75, 150), (1, 72, 257, 5, 7)])
def test_conv1x1_under_reserve(reserve, N, Cin, Cout, H, W, monkeypatch):
    tcb.test_conv1x1_gemm_fwd_dgrad("bf16x6", N, Cin, Cout, H, W, monkeypatch)


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(556, 4096, 25088), (556, 300, 1000), (300, 1024, 4105)])
def test_gemm_under_reserve(reserve, M, N, K, ak, bk):
    tlg.test_gemm_layouts(M, N, K, ak, bk, "bf16x6")


def test_masked_dgrad_and_determinism_under_reserve(reserve):
    """The fused dgrad epilogue on split-K tail tiles and the fixed-order reduces stay
    bit-repeatable under the reserve's plans."""
    from tlod.conv import conv_dgrad, conv_wgrad
    g = torch.Generator().manual_seed(7)
    gy = torch.randn(2, 512, 37, 75, generator=g).to(dev)
    w = (torch.randn(512, 512, 3, 3, generator=g) * 0.02).to(dev)
    m = torch.relu(torch.randn(2, 512, 37, 75, generator=g)).to(dev)
    a = conv_dgrad(gy, w, math="bf16x6", mask=m)
    assert torch.equal(a, conv_dgrad(gy, w, math="bf16x6") * (m > 0))
    x = torch.randn(2, 512, 37, 75, generator=g).to(dev)
    assert torch.equal(conv_wgrad(gy, x, 3, math="bf16x6"), conv_wgrad(gy, x, 3, math="bf16x6"))


def test_reserve_changes_the_plans():
    """The reserve is not a no-op: split-K workspaces of the conv / GEMM planners differ
    between 0 and 32 reserved CUs on shapes whose rounds depend on the slot count."""
    from tlod import _lib
    L = _lib.lib()
    queries = [
        lambda: L.tlod_conv_fwd_bs_workspace_bytes(2, 256, 150, 250, 256, 3, 6),
        lambda: L.tlod_conv_fwd_bs_workspace_bytes(2, 512, 37, 75, 512, 3, 6),
        lambda: L.tlod_conv_wgrad_bs_workspace_bytes(2, 256, 150, 250, 256, 3, 6),
        lambda: L.tlod_gemm_bs_workspace_bytes(556, 4096, 25088, 1, 0, 6),
        lambda: L.tlod_conv1x1_gemm_bs_workspace_bytes(2, 1024, 38, 75, 256, 0, 6),
    ]
    try:
        base = [q() for q in queries]
        _lib.check(L.tlod_set_cu_reserve(32), "set_cu_reserve")
        held = [q() for q in queries]
    finally:
        _lib.check(L.tlod_set_cu_reserve(0), "set_cu_reserve")
    assert [q() for q in queries] == base
    assert sum(a != b for a, b in zip(base, held)) >= 2, (base, held)


def test_reserve_argument_checked():
    from tlod import _lib
    L = _lib.lib()
    assert L.tlod_set_cu_reserve(-1) != 0
    assert L.tlod_set_cu_reserve(0) == 0
    y = F.relu(torch.ones(1, device=dev))  # the device still works after the rejected call
    assert float(y) == 1.0
