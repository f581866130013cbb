"""Parity of the HIP NMS / RoIAlign / RoIPool kernels with the CPU oracle (C ABI path).

Bars: NMS keep indices and RoIPool argmax bit-exact; RoIAlign / RoIPool forward values
bit-exact (the kernels restate the CUDA arithmetic with -ffp-contract=off); backward
values (atomic accumulation, order-dependent) within rtol 1e-5 / atol 1e-6.
"""
import numpy as np
import pytest
import torch

from helpers import anchor_grid_boxes, clustered_boxes, random_boxes, sorted_dets
from oracle import nms as onms
from oracle import roi as oroi

pytestmark = pytest.mark.gpu
dev = "cuda"


def _nms(d, thr, max_keep=0):
    from tlod.nms import nms
    k = nms(torch.from_numpy(d).to(dev), thr, max_keep=max_keep)
    return np.asarray([]) if isinstance(k, list) else k.cpu().numpy()


@pytest.mark.parametrize("n,thr,kind", [(12000, 0.7, "clustered"), (12000, 0.7, "random"),
                                        (6000, 0.7, "clustered"), (300, 0.3, "clustered"),
                                        (65, 0.5, "clustered"), (64, 0.5, "clustered"),
                                        (1, 0.7, "random"), (2000, 0.0, "random"),
                                        (3000, 1.0, "clustered"), (16384, 0.7, "clustered"),
                                        (20000, 0.6, "clustered")])
def test_nms_bit_exact(n, thr, kind):
    rng = np.random.default_rng(n + int(thr * 10))
    boxes = clustered_boxes(rng, n) if kind == "clustered" else random_boxes(rng, n)
    d = sorted_dets(boxes, rng)
    ref = onms.nms(d, thr)
    got = _nms(d, thr)
    assert got.dtype == np.int32
    np.testing.assert_array_equal(got, ref)


def test_nms_max_keep_and_duplicates():
    rng = np.random.default_rng(7)
    b = clustered_boxes(rng, 5000, clusters=400)
    b[100:200] = b[100]  # exact duplicates: IoU == 1
    d = sorted_dets(b, rng)
    for mk in (1, 63, 64, 65, 300, 2000):
        np.testing.assert_array_equal(_nms(d, 0.7, mk), onms.nms(d, 0.7, max_keep=mk))


@pytest.mark.parametrize("n,mk", [(12000, 2000), (6000, 300), (12000, 0), (4000, 65)])
def test_nms_anchor_grid_proposals(n, mk):
    """The proposal layer's regime (dense anchors, ~20-50 survivors per 64-box block, early
    stop at post_nms): exercises the scan's survivor-row fetches across many blocks."""
    rng = np.random.default_rng(n + mk)
    d = sorted_dets(anchor_grid_boxes(rng), rng)[:n]
    np.testing.assert_array_equal(_nms(d, 0.7, mk), onms.nms(d, 0.7, max_keep=mk or None))


def test_nms_empty():
    from tlod.nms import nms
    assert nms(torch.zeros((0, 5), device=dev), 0.7) == []


def _feat(rng, B=1, C=64, H=37, W=62):
    return rng.standard_normal((B, C, H, W)).astype(np.float32)


def _rois(rng, R, B=1, W=1000, H=600, edge=True):
    b = random_boxes(rng, R, W, H, 4, 500)
    if edge:  # malformed / out-of-image / tiny boxes
        b[0] = [W - 2, H - 2, W + 40, H + 40]
        b[1] = [-30, -30, 5, 5]
        b[2] = [100, 100, 90, 95]   # x2 < x1
        b[3] = [0, 0, 0, 0]
        b[4] = [10.5, 20.25, 10.5, 20.25]
    bi = rng.integers(0, B, R).astype(np.float32)
    return np.concatenate([bi[:, None], b], 1).astype(np.float32)


@pytest.mark.parametrize("B,C,H,W,R,ah,aw", [(1, 64, 37, 62, 128, 8, 8), (2, 32, 20, 30, 50, 8, 8),
                                             (1, 16, 9, 11, 40, 4, 6)])
def test_roi_align_fwd_bwd(B, C, H, W, R, ah, aw):
    from tlod.roi_align import RoIAlignFunction
    rng = np.random.default_rng(B * 100 + C)
    f = _feat(rng, B, C, H, W)
    r = _rois(rng, R, B, W * 16, H * 16)
    ft = torch.from_numpy(f).to(dev).requires_grad_(True)
    out = RoIAlignFunction.apply(ft, torch.from_numpy(r).to(dev), ah, aw, 1.0 / 16)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), oroi.roi_align_fwd(f, r, ah, aw, 1.0 / 16))
    g = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(dev))
    ref = oroi.roi_align_bwd(g, r, B, C, H, W, 1.0 / 16)
    np.testing.assert_allclose(ft.grad.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("path", ["gather", "atomic"])
@pytest.mark.parametrize("B,C,H,W,R", [(1, 512, 37, 62, 256), (1, 100, 37, 75, 300), (2, 64, 12, 16, 33),
                                       (2, 33, 37, 75, 556), (2, 8, 100, 120, 60)])
def test_roi_align_avg_fused(B, C, H, W, R, path, monkeypatch):
    """Odd C, RoIs of two images interleaved; (2, 33, 37, 75, 556) is the DAF step's RoI
    count on its base-feature map; backward through the default sorted-tap gather and the
    atomic kernels (TLOD_ROI_BWD_GATHER=0)."""
    from tlod.roi_align import RoIAlignAvg
    monkeypatch.setenv("TLOD_ROI_BWD_GATHER", "1" if path == "gather" else "0")
    rng = np.random.default_rng(R)
    f = _feat(rng, B, C, H, W)
    r = _rois(rng, R, B, W * 16, H * 16)
    ft = torch.from_numpy(f).to(dev).requires_grad_(True)
    out = RoIAlignAvg(7, 7, 1.0 / 16)(ft, torch.from_numpy(r).to(dev))
    assert out.shape == (R, C, 7, 7)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), oroi.roi_align_avg_fwd(f, r, 7, 7, 1.0 / 16))
    g = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(dev))
    ref = oroi.roi_align_avg_bwd(g, r, B, C, H, W, 1.0 / 16)
    np.testing.assert_allclose(ft.grad.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,C,H,W,R,P", [(2, 512, 37, 75, 556, 7), (1, 40, 20, 30, 90, 3),
                                         (2, 16, 6, 5, 17, 7), (1, 70, 20, 30, -300, 7)])
def test_roi_align_avg_bwd_gather(B, C, H, W, R, P, monkeypatch):
    """The gather backward (taps sorted by feature cell, no atomics) is deterministic — two
    calls bit-identical — and matches the oracle to 1e-5; (2, 16, 6, 5): RoIs past the map
    (invalid samples); R = -300: 300 copies of one small RoI, so a few cells take thousands
    of taps whose runs cross many 64-tap segments (the carry / fixup chain)."""
    from tlod.roi_align import RoIAlignAvg
    monkeypatch.setenv("TLOD_ROI_BWD_GATHER", "1")
    rng = np.random.default_rng(abs(R) + P)
    f = _feat(rng, B, C, H, W)
    atol = 1e-5
    if R < 0:
        r = np.tile(np.array([[0, 100.0, 90.0, 130.0, 121.0]], np.float32), (-R, 1))
        R = -R
        atol = 1e-4  # ~8k-term sums (partials ~10x the result) in another order than the oracle
    else:
        r = _rois(rng, R, B, W * 16 + 200, H * 16 + 200)
    g = rng.standard_normal((R, C, P, P)).astype(np.float32)

    def grad():
        ft = torch.from_numpy(f).to(dev).requires_grad_(True)
        out = RoIAlignAvg(P, P, 1.0 / 16)(ft, torch.from_numpy(r).to(dev))
        out.backward(torch.from_numpy(g).to(dev))
        return ft.grad.cpu().numpy()
    a, b = grad(), grad()
    np.testing.assert_array_equal(a, b)
    ref = oroi.roi_align_avg_bwd(g, r, B, C, H, W, 1.0 / 16)
    np.testing.assert_allclose(a, ref, rtol=1e-5, atol=atol)


@pytest.mark.parametrize("B,C,H,W,R,P", [(2, 1024, 38, 75, 600, 7), (1, 40, 20, 30, 90, 7),
                                         (2, 300, 12, 16, 33, 6), (2, 16, 6, 5, 17, 5),
                                         (1, 70, 20, 30, -300, 7), (1, 8, 10, 12, 5, 1)])
def test_roi_head_entry_matches_roi_align_avg(B, C, H, W, R, P, monkeypatch):
    """The ResNet RoI head's entry (tlod_roi_align_avg_s2_nhwc_*: bins (2i, 2j), channels-last)
    against the fused RoIAlignAvg -> permute -> stride-2 subsample it replaces, forward and
    backward bit for bit (both backwards on the sorted-tap gather: the same taps in the same
    order); even P leaves the last sample row / column without a bin; R = -300: one small
    RoI 300 times (runs across many tap segments); (2, 16, 6, 5): RoIs past the map."""
    from tlod.roi_align import RoIAlignAvgFunction, roi_align_avg_s2_nhwc
    monkeypatch.setenv("TLOD_ROI_BWD_GATHER", "1")
    rng = np.random.default_rng(abs(R) + P + C)
    f = torch.from_numpy(_feat(rng, B, C, H, W)).to(dev)
    if R < 0:
        r = np.tile(np.array([[0, 100.0, 90.0, 130.0, 121.0]], np.float32), (-R, 1))
        R = -R
    else:
        r = _rois(rng, R, B, W * 16 + 200, H * 16 + 200)
    rt = torch.from_numpy(r).to(dev)
    Q = (P + 1) // 2
    g = torch.from_numpy(rng.standard_normal((R, Q, Q, C)).astype(np.float32)).to(dev)
    fa = f.clone().requires_grad_(True)
    got = roi_align_avg_s2_nhwc(fa, rt, P, P, 1.0 / 16)
    fb = f.clone().requires_grad_(True)
    ref = RoIAlignAvgFunction.apply(fb, rt, P, P, 1.0 / 16).permute(0, 2, 3, 1)[:, ::2, ::2, :]
    assert got.shape == (R, Q, Q, C) and got.is_contiguous()
    assert torch.equal(got, ref)
    got.backward(g)
    ref.backward(g)
    assert torch.equal(fa.grad, fb.grad)


@pytest.mark.parametrize("B,C,H,W,R", [(1, 64, 37, 62, 128), (2, 16, 20, 25, 40)])
def test_roi_pool_fwd_bwd(B, C, H, W, R):
    from tlod.roi_pool import roi_pool_with_argmax
    rng = np.random.default_rng(R + C)
    f = _feat(rng, B, C, H, W)
    r = _rois(rng, R, B, W * 16, H * 16)
    ft = torch.from_numpy(f).to(dev).requires_grad_(True)
    out, arg = roi_pool_with_argmax(ft, torch.from_numpy(r).to(dev), 7, 7, 1.0 / 16)
    ro, ra = oroi.roi_pool_fwd(f, r, 7, 7, 1.0 / 16)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ro)
    np.testing.assert_array_equal(arg.cpu().numpy(), ra)
    g = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(dev))
    ref = oroi.roi_pool_bwd(g, ra, r, B, C, H, W, 1.0 / 16)
    np.testing.assert_allclose(ft.grad.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


def test_roi_ops_empty_rois():
    from tlod.roi_align import RoIAlignAvg
    f = torch.randn(1, 8, 10, 10, device=dev)
    out = RoIAlignAvg(7, 7, 1.0 / 16)(f, torch.zeros((0, 5), device=dev))
    assert out.shape == (0, 8, 7, 7)
