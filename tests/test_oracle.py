"""CPU checks of the oracle itself: pinned by the reference's only known-answer vector
(generate_anchors.py:29-37) and by internal consistency properties; golden fixtures
under tests/golden are regenerated and compared by test_golden.py."""
import numpy as np

from oracle.boxes import bbox_overlaps, bbox_transform, bbox_transform_inv, generate_anchors
from oracle.nms import nms
from oracle import roi as oroi

# generate_anchors.py:29-37 (MATLAB, 1-based); the Python restatement yields value - 1.
MATLAB_KAT = np.array([[-83, -39, 100, 56], [-175, -87, 192, 104], [-359, -183, 376, 200],
                       [-55, -55, 72, 72], [-119, -119, 136, 136], [-247, -247, 264, 264],
                       [-35, -79, 52, 96], [-79, -167, 96, 184], [-167, -343, 184, 360]],
                      np.float32)


def test_anchor_known_answer():
    np.testing.assert_array_equal(generate_anchors(), MATLAB_KAT - 1)


def test_anchor_scale4_row():
    a = generate_anchors(scales=(4, 8, 16, 32))
    assert a.shape == (12, 4)
    np.testing.assert_array_equal(a[0], [-38, -16, 53, 31])  # SURVEY §8c hand-derived row


def test_product_anchors_match_oracle():
    from tlod.rpn.anchors import generate_anchors as prod
    for sc in [(8, 16, 32), (4, 8, 16, 32)]:
        np.testing.assert_array_equal(prod(scales=sc).astype(np.float32), generate_anchors(scales=sc))


def test_transform_roundtrip():
    rng = np.random.default_rng(0)
    ex = rng.uniform(0, 500, (100, 4)).astype(np.float32)
    ex[:, 2:] += ex[:, :2] + 10
    gt = ex + rng.normal(0, 5, ex.shape).astype(np.float32)
    d = bbox_transform(ex, gt)
    back = bbox_transform_inv(ex, d)
    # "+1" widths: inv(transform(gt)) = (x1, y1, x2 + 1, y2 + 1)
    np.testing.assert_allclose(back[:, :2], gt[:, :2], atol=2e-3)
    np.testing.assert_allclose(back[:, 2:], gt[:, 2:] + 1, atol=2e-3)


def test_overlaps_masks():
    a = np.array([[0, 0, 9, 9], [5, 5, 5, 5]], np.float32)   # second: zero-area anchor
    g = np.array([[0, 0, 9, 9, 1], [0, 0, 0, 0, 0]], np.float32)  # second: zero gt
    ov = bbox_overlaps(a, g)
    assert ov[0, 0] == 1 and ov[0, 1] == 0 and (ov[1] == -1).all()


def test_nms_properties():
    rng = np.random.default_rng(1)
    b = rng.uniform(0, 300, (500, 4)).astype(np.float32)
    b[:, 2:] = b[:, :2] + rng.uniform(5, 80, (500, 2)).astype(np.float32)
    d = np.concatenate([b, np.linspace(1, 0, 500, dtype=np.float32)[:, None]], 1)
    k = nms(d, 0.5)
    assert k[0] == 0 and np.all(np.diff(k) > 0)
    kb = d[k, :4]
    from oracle.boxes import iou_pair_cuda
    for i in range(len(kb)):                      # survivors pairwise below threshold
        assert (iou_pair_cuda(kb[i], kb[i + 1:]) <= np.float32(0.5)).all()
    assert len(nms(d, 1.0)) == 500 and len(nms(d[:0], 0.5)) == 0


def test_roi_align_avg_shapes_and_linearity():
    rng = np.random.default_rng(2)
    f = rng.standard_normal((1, 4, 10, 12)).astype(np.float32)
    r = np.array([[0, 10, 10, 120, 90], [0, 0, 0, 15, 15]], np.float32)
    o = oroi.roi_align_avg_fwd(f, r, 7, 7, 1 / 16)
    assert o.shape == (2, 4, 7, 7)
    o2 = oroi.roi_align_avg_fwd(2 * f, r, 7, 7, 1 / 16)
    np.testing.assert_allclose(o2, 2 * o, rtol=1e-6)
    # adjoint: <A f, g> == <f, A^T g>
    g = rng.standard_normal(o.shape).astype(np.float32)
    gb = oroi.roi_align_avg_bwd(g, r, 1, 4, 10, 12, 1 / 16)
    np.testing.assert_allclose((o * g).sum(), (f * gb).sum(), rtol=1e-4)


def test_roi_pool_adjoint():
    rng = np.random.default_rng(3)
    f = rng.standard_normal((1, 3, 9, 9)).astype(np.float32)
    r = np.array([[0, 0, 0, 100, 100], [0, 16, 32, 64, 128]], np.float32)
    o, a = oroi.roi_pool_fwd(f, r, 7, 7, 1 / 16)
    g = rng.standard_normal(o.shape).astype(np.float32)
    gb = oroi.roi_pool_bwd(g, a, r, 1, 3, 9, 9, 1 / 16)
    np.testing.assert_allclose((o * g).sum(), (f * gb).sum(), rtol=1e-4)


def test_drm_chunks_is_cropped_pixel_unshuffle():
    """The literal DRM restatement (lib/MAF/drm.py:23-40) equals pixel_unshuffle of the
    map cropped to whole s x s blocks: channel c*s*s + i*s + j <- (h*s + i, w*s + j)."""
    import torch
    import torch.nn.functional as F
    from oracle.maf_step import drm_chunks
    x = torch.randn(2, 5, 11, 14)
    for s in (2, 3, 4):
        Ho, Wo = 11 // s, 14 // s
        ref = F.pixel_unshuffle(x[:, :, :Ho * s, :Wo * s], s)
        assert torch.equal(drm_chunks(x, s), ref)


def test_oracle_steps_run_on_cpu():
    """The step oracles (test infrastructure) run end to end on a tiny batch, including the
    fp64 run and the activation-pattern record / force machinery the GPU tests use."""
    import copy

    import torch

    from helpers import record_pattern, run_in_pattern
    from oracle.daf_step import OracleDAF, synthetic_batch, total_loss
    torch.manual_seed(0)
    o = OracleDAF(dropout=0.0).train()
    b = synthetic_batch(96, 128, seed=3)
    own = record_pattern(o, lambda: total_loss(o(b, np.random.RandomState(3))).backward())
    assert "base.11" in own and "ip1" in own and len(own["base.11"]) == 2
    o64 = copy.deepcopy(o).double()
    b64 = tuple(t.double() if t.is_floating_point() else t for t in b)
    run_in_pattern(o64, own, lambda: total_loss(o64(b64, np.random.RandomState(3))).backward())
    g32 = dict(o.named_parameters())
    for k, p in o64.named_parameters():
        if p.grad is not None:
            e = float((g32[k].grad.double() - p.grad).norm() / max(float(p.grad.norm()), 1e-30))
            assert e < 1e-4, (k, e)
