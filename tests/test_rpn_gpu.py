"""Parity of the on-device proposal layer, anchor-target and proposal-target layers with
the oracle (oracle/rpn.py), at the DAF VGG16 canonical sizes.

Bars: integer outputs (NMS order, labels, sampled indices) bit-exact given the same
decoded boxes and the same numpy draws (replay mode); float outputs that go through
expf/logf (decode, regression targets) within rtol 2e-6 (library ulp differences).
"""
import numpy as np
import pytest
import torch

from helpers import gt_set, rpn_outputs
from oracle import rpn as orpn
from oracle.boxes import generate_anchors
from oracle.nms import nms as onms

pytestmark = pytest.mark.gpu
dev = "cuda"
BASE = generate_anchors(scales=np.array([4, 8, 16, 32]), ratios=np.array([0.5, 1, 2]))


@pytest.mark.parametrize("H,W,pre,post,thr", [(37, 62, 12000, 2000, 0.7), (37, 75, 6000, 300, 0.7),
                                              (10, 12, 12000, 2000, 0.7), (37, 75, 12000, 2000, 0.7)])
def test_proposal_layer(H, W, pre, post, thr):
    from tlod.rpn.proposal import proposal
    rng = np.random.default_rng(H * W + pre)
    A = BASE.shape[0]
    prob, deltas = rpn_outputs(rng, 1, A, H, W)
    im_info = np.array([[H * 16, W * 16, 1.0]], np.float32)
    t = lambda x: torch.from_numpy(x).to(dev)
    rois, props = proposal(t(prob), t(deltas), t(im_info), t(BASE), 16, pre, post, thr,
                           return_props=True)
    scores, oprops = orpn.decode_clip(prob, deltas, im_info, BASE, 16)
    gp = props.cpu().numpy()
    np.testing.assert_allclose(gp, oprops, rtol=2e-6, atol=1e-4)
    # NMS/order parity on the device-decoded boxes (isolates expf ulp differences)
    order = np.argsort(-scores[0], kind="stable")[:pre]
    keep = onms(np.concatenate([gp[0][order], scores[0][order, None]], 1), thr, max_keep=post)
    exp = np.zeros((post, 5), np.float32)
    exp[:len(keep), 1:] = gp[0][order][keep]
    np.testing.assert_array_equal(rois.cpu().numpy()[0], exp)


def test_proposal_layer_batch2_matches_oracle():
    from tlod.rpn.proposal import proposal
    rng = np.random.default_rng(5)
    A, H, W = 12, 20, 30
    prob, deltas = rpn_outputs(rng, 2, A, H, W, delta_scale=0.0)  # exp(0)=1: decode exact
    im_info = np.array([[320, 480, 1.0], [300, 400, 1.0]], np.float32)
    t = lambda x: torch.from_numpy(x).to(dev)
    rois = proposal(t(prob), t(deltas), t(im_info), t(BASE), 16, 3000, 500, 0.7)
    ref = orpn.proposal_layer(prob, deltas, im_info, BASE, 16, 3000, 500, 0.7)
    np.testing.assert_array_equal(rois.cpu().numpy(), ref)


def _anchor_case(seed, H, W, G, B=1):
    rng = np.random.default_rng(seed)
    gts = np.stack([gt_set(rng, G=G, W=W * 16, H=H * 16) for _ in range(B)])
    im_info = np.array([[H * 16, W * 16, 1.0]] * B, np.float32)
    return gts, im_info


@pytest.mark.parametrize("seed,H,W,G,B", [(0, 37, 62, 8, 1), (1, 37, 75, 8, 1), (2, 37, 75, 30, 1),
                                          (3, 20, 30, 3, 2), (4, 37, 62, 1, 1)])
def test_anchor_target_replay_bit_exact(seed, H, W, G, B):
    from tlod.rpn.anchor_target import anchor_target, rpn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    gts, im_info = _anchor_case(seed, H, W, G, B)
    rec = orpn.Recorder(seed)
    ref = orpn.anchor_target(H, W, gts, im_info, BASE, 16, rec)
    draws = iter([x for _, x in rec.log])

    class Replay:
        def permutation(self, n):
            p = next(draws)
            assert len(p) == n
            return p

    t = lambda x: torch.from_numpy(x).to(dev)
    got = anchor_target(t(BASE), H, W, 16, t(gts), t(im_info), rpn_cfg_struct(), rng=Replay())
    names = ["labels", "targets", "inside", "outside"]
    for name, g, r in zip(names, got, ref):
        g = g.cpu().numpy()
        if name == "targets":
            np.testing.assert_allclose(g, r, rtol=2e-6, atol=2e-6, err_msg=name)
        else:
            np.testing.assert_array_equal(g, r, err_msg=name)


def test_anchor_target_device_rng_distribution():
    """Production mode: exact fg/bg budget, only subsamples pre-sampling candidates."""
    from tlod.rpn.anchor_target import anchor_target, rpn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    H, W = 37, 75
    gts, im_info = _anchor_case(11, H, W, 8)
    t = lambda x: torch.from_numpy(x).to(dev)
    labs = [anchor_target(t(BASE), H, W, 16, t(gts), t(im_info), rpn_cfg_struct(), seed=s)[0]
            .cpu().numpy().ravel() for s in range(4)]
    # replay with the identity "permutation" gives the candidate sets
    full = orpn.anchor_target(H, W, gts, im_info, BASE, 16,
                              type("N", (), {"permutation": lambda self, n: np.arange(n)})())[0].ravel()
    for l in labs:
        assert (l == 1).sum() + (l == 0).sum() == 256
        assert (l == 1).sum() <= 128
    assert not all(np.array_equal(labs[0], l) for l in labs[1:])
    del full


def _rng_key(seed, stream, idx):
    """(rng_u64(seed, stream, idx) >> 32) of csrc/common.h (splitmix64 twice), in numpy."""
    def mix(z):
        z = z + np.uint64(0x9e3779b97f4a7c15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))
    with np.errstate(over="ignore"):
        base = mix(np.array([seed], np.uint64) ^ (np.array([stream], np.uint64) *
                                                  np.uint64(0xd1b54a32d192ed03)))
        return (mix(base + idx.astype(np.uint64)) >> np.uint64(32)).astype(np.uint32)


@pytest.mark.parametrize("H,W,seed", [(37, 75, 5), (38, 75, 77), (20, 30, 3), (50, 100, 9)])
def test_anchor_target_device_rng_exact_subset(H, W, seed):
    """Production mode pinned exactly: the kept fg / bg anchors are the candidates whose
    (key, anchor index) pairs are NOT among the m smallest, key = rng_u64(seed, 2b (fg) /
    2b + 1 (bg), anchor) >> 32 — restated here in numpy.  (37, 75), (38, 75): the
    LDS-key kernel (N = 33300 / 34200 anchors); (50, 100): N = 60000, the list kernel."""
    from tlod.rpn.anchor_target import anchor_target, rpn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    rng = np.random.default_rng(seed)
    gts = gt_set(rng, G=50, W=W * 16, H=H * 16)[None]
    gts[0, :, 2:4] = np.maximum(gts[0, :, 2:4], gts[0, :, 0:2] + 200)  # big boxes: many fg
    gts[0, :, 2] = np.minimum(gts[0, :, 2], W * 16 - 1)
    gts[0, :, 3] = np.minimum(gts[0, :, 3], H * 16 - 1)
    im_info = np.array([[H * 16, W * 16, 1.0]], np.float32)
    ident = type("N", (), {"permutation": lambda self, n: np.arange(n)})()
    cfg = dict(orpn.DEFAULT_RPN)
    cfg["batch"] = 10 ** 9  # no subsampling: the candidates
    cand = orpn.anchor_target(H, W, gts, im_info, BASE, 16, ident, cfg)[0].ravel()
    t = lambda x: torch.from_numpy(x).to(dev)
    lab = anchor_target(t(BASE), H, W, 16, t(gts), t(im_info), rpn_cfg_struct(),
                        seed=seed)[0].reshape(-1).cpu().numpy()
    A, HW = BASE.shape[0], H * W
    p = np.arange(A * HW)
    idx = (p % HW) * A + p // HW  # output (a, h, w) -> the kernels' anchor index (h, w, a)
    exp = cand.copy()
    fg = np.nonzero(cand == 1)[0]
    m_fg = max(0, len(fg) - 128)
    k = _rng_key(seed, 0, idx[fg])
    exp[fg[np.lexsort((idx[fg], k))[:m_fg]]] = -1
    bg = np.nonzero(cand == 0)[0]
    m_bg = len(bg) - (256 - min(len(fg), 128))
    assert m_bg > 0
    k = _rng_key(seed, 1, idx[bg])
    exp[bg[np.lexsort((idx[bg], k))[:m_bg]]] = -1
    np.testing.assert_array_equal(lab, exp)


@pytest.mark.parametrize("seed,G,R", [(0, 8, 2000), (1, 30, 2000), (2, 2, 300), (3, 8, 128)])
def test_proposal_target_replay_bit_exact(seed, G, R):
    from tlod.rpn.proposal_target import proposal_target, rcnn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    rng = np.random.default_rng(seed)
    gt = gt_set(rng, G=G)[None]
    # proposals: jittered gts + random boxes + zero padding rows
    from helpers import random_boxes
    n_real = R - 37
    near = gt[0, rng.integers(0, G, n_real // 2), :4] + rng.normal(0, 20, (n_real // 2, 4))
    far = random_boxes(rng, n_real - n_real // 2)
    boxes = np.concatenate([near, far]).astype(np.float32)
    boxes[:, 2:] = np.maximum(boxes[:, 2:], boxes[:, :2] + 1)
    rois = np.zeros((1, R, 5), np.float32)
    rois[0, :n_real, 1:] = np.clip(boxes, 0, 999)
    rec = orpn.Recorder(seed + 100)
    ref = orpn.proposal_target(rois, gt, rec)
    draws = iter([x for _, x in rec.log])

    class Replay:
        def permutation(self, n):
            p = next(draws)
            assert len(p) == n
            return p

        def rand(self, n):
            u = next(draws)
            assert len(u) == n
            return u

    t = lambda x: torch.from_numpy(x).to(dev)
    got = proposal_target(t(rois), t(gt), rcnn_cfg_struct(), rng=Replay())
    for name, g, r in zip(["rois", "labels", "targets", "inside", "outside"], got, ref):
        g = g.cpu().numpy()
        if name == "targets":
            np.testing.assert_allclose(g, r, rtol=2e-6, atol=2e-6, err_msg=name)
        else:
            np.testing.assert_array_equal(g, r, err_msg=name)


def test_proposal_target_device_rng():
    from tlod.rpn.proposal_target import proposal_target, rcnn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    rng = np.random.default_rng(9)
    gt = gt_set(rng, G=8)[None]
    rois = np.zeros((1, 2000, 5), np.float32)
    from helpers import random_boxes
    rois[0, :, 1:] = random_boxes(rng, 2000)
    t = lambda x: torch.from_numpy(x).to(dev)
    r, lab, tg, iw, ow = proposal_target(t(rois), t(gt), rcnn_cfg_struct(), seed=123)
    lab = lab.cpu().numpy()[0]
    nfg = int((lab > 0).sum())
    assert 8 <= nfg <= 64            # every gt is itself a fg candidate
    assert (lab[nfg:] == 0).all()    # fg first, then bg
    assert np.all(iw.cpu().numpy()[0][lab > 0] == 1) and np.all(iw.cpu().numpy()[0][lab == 0] == 0)


def test_device_subset_sampling_is_uniform():
    """the production sampler (block_random_subset: per-candidate hashed
    keys, radix-selected smallest k) picks every candidate with the same probability, as
    the reference's np.random.permutation(n)[:k] does (anchor_target_layer.py:123-145).
    Over 1200 seeds each fg / bg candidate's selection count stays within 5 sigma of the
    binomial mean k/n."""
    from tlod.rpn.anchor_target import anchor_target, rpn_cfg_struct
    from tlod.config import setup_training_cfg
    setup_training_cfg("vgg16")
    H, W = 37, 75
    rng = np.random.default_rng(21)
    gts = gt_set(rng, G=50, W=W * 16, H=H * 16)[None]
    gts[0, :, 2:4] = np.maximum(gts[0, :, 2:4], gts[0, :, 0:2] + 200)  # big boxes: many fg
    gts[0, :, 2] = np.minimum(gts[0, :, 2], W * 16 - 1)
    gts[0, :, 3] = np.minimum(gts[0, :, 3], H * 16 - 1)
    im_info = np.array([[H * 16, W * 16, 1.0]], np.float32)
    ident = type("N", (), {"permutation": lambda self, n: np.arange(n)})()
    full = orpn.anchor_target(H, W, gts, im_info, BASE, 16, ident)[0].ravel()
    # the candidates before subsampling: with the identity "permutation" the reference keeps
    # the first k; recompute the candidate sets from the pre-sampling rules instead
    cfg = dict(orpn.DEFAULT_RPN)
    cfg["batch"] = 10 ** 9  # no subsampling: every candidate keeps its label
    cand = orpn.anchor_target(H, W, gts, im_info, BASE, 16, ident, cfg)[0].ravel()
    fg_c, bg_c = np.nonzero(cand == 1)[0], np.nonzero(cand == 0)[0]
    assert len(fg_c) > 128 and len(bg_c) > 256, (len(fg_c), len(bg_c))
    t = lambda x: torch.from_numpy(x).to(dev)
    seeds = 1200
    cnt = torch.zeros(full.size, dtype=torch.float64, device=dev)
    for s in range(seeds):
        lab = anchor_target(t(BASE), H, W, 16, t(gts), t(im_info), rpn_cfg_struct(), seed=s)[0]
        cnt += (lab.reshape(-1) >= 0).double()
    cnt = cnt.cpu().numpy()
    for cands, k in ((fg_c, 128), (bg_c, 256 - 128)):
        p = k / len(cands)
        mu, sd = seeds * p, np.sqrt(seeds * p * (1 - p))
        z = np.abs(cnt[cands] - mu) / sd
        assert z.max() < 5.0, (len(cands), k, float(z.max()))
        outside = np.setdiff1d(np.arange(full.size), np.concatenate([fg_c, bg_c]))
    assert cnt[outside].max() == 0
