"""Synthetic inputs shared by the tests (seeded, reference-shaped)."""
import numpy as np


def random_boxes(rng, n, W=1000, H=600, min_wh=8, max_wh=300):
    x1 = rng.uniform(0, W - min_wh, n)
    y1 = rng.uniform(0, H - min_wh, n)
    w = rng.uniform(min_wh, max_wh, n)
    h = rng.uniform(min_wh, max_wh, n)
    x2 = np.minimum(x1 + w, W - 1)
    y2 = np.minimum(y1 + h, H - 1)
    return np.stack([x1, y1, x2, y2], 1).astype(np.float32)


def clustered_boxes(rng, n, W=1000, H=600, clusters=40):
    """Heavily overlapping boxes (exercises the NMS suppression paths)."""
    c = random_boxes(rng, clusters, W, H, 32, 300)
    idx = rng.integers(0, clusters, n)
    jitter = rng.normal(0, 6, (n, 4)).astype(np.float32)
    b = c[idx] + jitter
    b[:, 2] = np.maximum(b[:, 2], b[:, 0] + 1)
    b[:, 3] = np.maximum(b[:, 3], b[:, 1] + 1)
    return np.clip(b, 0, [W - 1, H - 1, W - 1, H - 1]).astype(np.float32)


def sorted_dets(boxes, rng):
    s = rng.permutation(len(boxes)).astype(np.float32) / max(len(boxes), 1)  # tie-free
    order = np.argsort(-s, kind="stable")
    return np.concatenate([boxes[order], s[order, None]], 1).astype(np.float32)


def gt_set(rng, G=8, pad=50, W=1000, H=600, ncls=8):
    """G real gt boxes (x1 in [0,W-64), size 32..400, clipped), class 1..ncls, zero-padded."""
    gt = np.zeros((pad, 5), np.float32)
    x1 = rng.uniform(0, W - 64, G)
    y1 = rng.uniform(0, H - 64, G)
    w = rng.uniform(32, 400, G)
    h = rng.uniform(32, 400, G)
    gt[:G, 0] = np.floor(x1)
    gt[:G, 1] = np.floor(y1)
    gt[:G, 2] = np.minimum(np.floor(x1 + w), W - 1)
    gt[:G, 3] = np.minimum(np.floor(y1 + h), H - 1)
    gt[:G, 4] = rng.integers(1, ncls + 1, G)
    return gt


def rpn_outputs(rng, B, A, H, W, delta_scale=0.2):
    """Synthetic RPN head outputs: softmax'd cls prob (B,2A,H,W), deltas (B,4A,H,W)."""
    logits = rng.normal(0, 1, (B, 2, A, H, W)).astype(np.float32)
    e = np.exp(logits - logits.max(1, keepdims=True))
    p = (e / e.sum(1, keepdims=True)).astype(np.float32)
    prob = p.reshape(B, 2 * A, H, W)
    deltas = (rng.normal(0, delta_scale, (B, 4 * A, H, W))).astype(np.float32)
    return prob, deltas


def grad_errors(dev_named_params, o32, o64):
    """Normwise relative error of each trainable gradient against the fp64 oracle run, for
    the device (split-bf16 / fp32 kernels) and for the fp32 CPU oracle itself:
    {name: (err_device, err_fp32_oracle)}."""
    import torch
    gp = dict(dev_named_params)
    g64 = dict(o64.named_parameters())
    out = {}
    for k, p in o32.named_parameters():
        if not p.requires_grad or p.grad is None:
            continue
        ref = g64[k].grad.double()
        den = max(float(ref.norm()), 1e-30)
        ed = float((gp[k].grad.detach().double().cpu() - ref).norm()) / den
        e32 = float((p.grad.double() - ref).norm()) / den
        out[k] = (ed, e32)
    assert out, "no gradients compared"
    _ = torch
    return out


def assert_grad_bar(errs, factor=2.0, floor=2e-6):
    """the device gradient's error against fp64 is at most ``factor`` x
    the fp32 CPU oracle's own error against fp64 (with an fp32-roundoff floor, for
    gradients the fp32 oracle happens to reproduce almost exactly)."""
    bad = {k: v for k, v in errs.items() if v[0] > factor * max(v[1], floor)}
    assert not bad, {"violations": bad,
                     "worst_ratio": max(v[0] / max(v[1], floor) for v in errs.values())}
