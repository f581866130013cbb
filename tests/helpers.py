"""Synthetic inputs shared by the tests (seeded, reference-shaped)."""
import os

import numpy as np
import torch


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


def anchor_grid_boxes(rng, H=37, W=75, stride=16, imh=600, imw=1200, jitter=2.0):
    """RPN-like proposals: the 9 anchors (scales 8/16/32, ratios 0.5/1/2) at every feature
    cell of a 600x1200 image, slightly jittered and clipped (what the proposal layer's NMS
    sees from a fresh RPN: dense, heavily overlapping, ~1 in 3 kept at IoU 0.7)."""
    base = []
    for r in (0.5, 1.0, 2.0):
        for sc in (8, 16, 32):
            w, h = 16 * sc / np.sqrt(r), 16 * sc * np.sqrt(r)
            base.append([7.5 - 0.5 * (w - 1), 7.5 - 0.5 * (h - 1), 7.5 + 0.5 * (w - 1),
                         7.5 + 0.5 * (h - 1)])
    ys, xs = np.meshgrid(np.arange(H) * stride, np.arange(W) * stride, indexing="ij")
    sh = np.stack([xs, ys, xs, ys], -1).reshape(-1, 1, 4)
    b = (sh + np.array(base)[None]).reshape(-1, 4) + rng.normal(0, jitter, (H * W * 9, 4))
    b[:, 0::2] = np.clip(b[:, 0::2], 0, imw - 1)
    b[:, 1::2] = np.clip(b[:, 1::2], 0, imh - 1)
    b[:, 2] = np.maximum(b[:, 2], b[:, 0])
    b[:, 3] = np.maximum(b[:, 3], b[:, 1])
    return b.astype(np.float32)


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


def grad_errors(dev_named_params, o32, o64, o64_own=None):
    """Normwise relative error of each trainable gradient against an fp64 oracle run, for
    the device (split-bf16 / fp32 kernels; reference o64, evaluated in the device's
    activation pattern) and for the fp32 CPU oracle itself (reference o64_own, in the fp32
    oracle's own pattern; default o64): {name: (err_device, err_fp32_oracle)}."""
    gp = dict(dev_named_params)
    g64 = dict(o64.named_parameters())
    g64o = dict((o64_own or o64).named_parameters())
    out = {}
    for k, p in o32.named_parameters():
        if not p.requires_grad or p.grad is None:
            continue
        ref, refo = g64[k].grad.double(), g64o[k].grad.double()
        ed = float((gp[k].grad.detach().double().cpu() - ref).norm()) / max(float(ref.norm()), 1e-30)
        e32 = float((p.grad.double() - refo).norm()) / max(float(refo.norm()), 1e-30)
        out[k] = (ed, e32)
    assert out, "no gradients compared"
    return out


def assert_grad_bar(errs, factor=2.0, floor=2e-6):
    """the device gradient's error against fp64 is at most ``factor`` x
    the fp32 CPU oracle's own error against fp64 (with an fp32-roundoff floor, for
    gradients the fp32 oracle happens to reproduce almost exactly)."""
    bad = {k: v for k, v in errs.items() if v[0] > factor * max(v[1], floor)}
    assert not bad, {"violations": bad,
                     "worst_ratio": max(v[0] / max(v[1], floor) for v in errs.values())}


# ---------------------------------------------------------------- activation patterns
# The gradient of a ReLU / max-pool network is piecewise: a pre-activation within rounding
# of 0 (or a near-tied pool window) can land on different sides in two runs, and the
# gradients then differ by O(1) in that unit — a property of the function, not an
# arithmetic error.  The fp64 references of the gradient bars are therefore evaluated in
# the activation pattern of the run they judge: the device's (from tlod's act_tap
# instrumentation) or the fp32 oracle's own (recorded by oracle.daf_step.forced_relu).
VGG_TRAINABLE_CONVS = (10, 12, 14, 17, 19, 21, 24, 26, 28)
VGG_POOL_AFTER = {14: 16, 21: 23}  # conv index -> the max-pool layer index after it


def arm_taps(m):
    """Attach act_tap lists to every trainable activation site of a device DAF / MAF / ATF
    model (VGG16 or ResNet101).  Returns {oracle site: (list, kind)}; kind says how the
    device's batched calls split into the oracle's per-image / per-RoI-set calls:
      "map"  — batch entries of a feature map (source first), "pool" likewise plus the
               max-pool argmax of the map, "head" — RoI rows of the detection head
               (fc6 / fc7 / ResNet layer4), "ins" — RoI rows of the instance discriminator.
    Site names follow the oracle: base.{relu index} (VGG), base.{i}.{block}.r1..r3
    (ResNet layer2 / layer3), top.0.{block}.r1..r3 (ResNet layer4 head), base_t.* (ATF's
    t branch), rpn, fc6, fc7, ida / ida3 / ida4 (image DA), drm3 / drm4 (MAF DRM), ip1, ip2."""
    from tlod.detector.resnet import Bottleneck
    taps = {}

    def add(site, mod, kind):
        mod.act_tap = []
        taps[site] = (mod.act_tap, kind)

    def backbone(base, prefix):
        if any(isinstance(x, Bottleneck) for x in base.modules()):
            for i, layer in enumerate(base):
                if not isinstance(layer, torch.nn.Sequential):
                    continue
                for j, blk in enumerate(layer):
                    if not any(p.requires_grad for p in blk.parameters()):
                        continue  # frozen layer1: no gradient flows through it
                    blk.act_tap = {"r1": [], "r2": [], "r3": []}
                    for r in ("r1", "r2", "r3"):
                        taps[f"{prefix}.{i}.{j}.{r}"] = (blk.act_tap[r], "head" if prefix == "top"
                                                         else "map")
            return
        for i in VGG_TRAINABLE_CONVS:
            add(f"{prefix}.{i + 1}", base[i], "map")
            if i in VGG_POOL_AFTER:
                taps[f"{prefix}.{VGG_POOL_AFTER[i]}"] = (base[i].act_tap, "pool")

    backbone(m.RCNN_base, "base")
    if hasattr(m, "RCNN_base_t"):
        backbone(m.RCNN_base_t, "base_t")
    if any(isinstance(x, Bottleneck) for x in m.RCNN_top.modules()):
        backbone(m.RCNN_top, "top")
    else:
        add("fc6", m.RCNN_top[0], "head")
        add("fc7", m.RCNN_top[3], "head")
    add("rpn", m.RCNN_rpn.RPN_Conv, "map")
    if not hasattr(m, "RCNN_imageDA"):  # source-only Faster R-CNN
        return taps
    add("ida", m.RCNN_imageDA.Conv1, "map")
    for lvl in (3, 4):
        h = getattr(m, f"RCNN_imageDA_{lvl}", None)
        if h is not None:
            add(f"ida{lvl}", h.Conv1, "map")
            if hasattr(h, "DRM"):
                add(f"drm{lvl}", h.DRM.conv_low_dim, "map")
    add("ip1", m.RCNN_instanceDA.dc_ip1, "ins")
    add("ip2", m.RCNN_instanceDA.dc_ip2, "ins")
    return taps


def arm_device_taps(m):
    return arm_taps(m)


def device_forced(taps, n_rows=None):
    """Oracle ``forced`` dict (site -> per-call masks / pool indices) from the device taps.
    Batched device tensors are split into the oracle's per-image calls (source first):
    maps by batch entry; RoI rows by ``n_rows`` — an int (split point of the head and the
    instance discriminator rows, DAF / MAF), a dict {"head": [sizes], "ins": [sizes]}
    (ATF's four RoI sets), or None (one call)."""
    import torch.nn.functional as F

    def sizes(kind):
        if isinstance(n_rows, dict):
            return n_rows[kind]
        return None if n_rows is None else [n_rows]

    def mask(t):
        return t if t.dtype == torch.bool else t > 0

    forced = {}
    for site, (lst, kind) in taps.items():
        if not lst:
            continue
        parts = []
        if kind in ("map", "pool"):
            for t in lst:
                t = t.detach().cpu()
                parts += [t[i:i + 1] for i in range(t.shape[0])]
        else:
            t = torch.cat([x.detach().cpu() for x in lst], 0)
            sz = sizes(kind)
            if sz is None:
                parts = [t]
            else:
                sz = list(sz)
                if sum(sz) < t.shape[0]:
                    sz.append(t.shape[0] - sum(sz))
                parts = list(torch.split(t, sz, 0))
        if kind == "pool":
            forced[site] = [F.max_pool2d(p, 2, 2, return_indices=True)[1] for p in parts]
        else:
            forced[site] = [mask(p) for p in parts]
    return forced


def run_in_pattern(o64, forced, fn):
    """Run fn() (an fp64 oracle forward + backward) with the oracle's sites forced."""
    o64.forced.clear()
    o64.forced.update({k: list(v) for k, v in forced.items()})
    try:
        return fn()
    finally:
        left = {k: len(v) for k, v in o64.forced.items() if k != "__record__" and v}
        o64.forced.clear()
        assert not left, f"unused forced masks: {left}"


def record_pattern(o32, fn):
    """Run fn() on the fp32 oracle while recording its own masks / pool indices."""
    o32.forced.clear()
    o32.forced["__record__"] = {}
    try:
        fn()
        return o32.forced["__record__"]
    finally:
        o32.forced.clear()


def pattern_grad_bar(m, o, run, cpu_batch, taps, n_rows, own32, factor=2.0, floor=2e-5):
    """The gradient bar of the step tests, in matched activation patterns.

    Three fp32 gradient sets are each compared with an fp64 run of the same step (same
    weights, RoIs and replayed draws) evaluated in their own activation pattern:
      device  — tlod on the MI355X (split-bf16 MFMA convs / GEMMs, fused kernels);
      cpu32   — the oracle in torch-CPU fp32 (oneDNN / MKL: pairwise-blocked sums);
      gpu32   — the same oracle with its conv / linear on this GPU in fp32 (MIOpen /
                hipBLASLt: the arithmetic the reference's PyTorch-CUDA path uses here).
    Bar: every parameter's device error <= max(factor x max(cpu32, gpu32), floor), floor =
    2e-5 normwise (50x inside north_star's 1e-3).  The floor is what the device needs: its
    split-bf16 MFMA path carries a small coherent shrink (~-6e-8 relative per conv layer
    through VGG16, none with the f32 MFMA) that the input-gradient chain
    compounds: conv3_1's gradients end at 1e-5 at most, where the fp32 references stay at
    2e-7..1.5e-6 — the printed ratios keep that gap visible.  ``run(model, batch)`` returns the oracle's total
    loss; ``own32`` is the cpu32 run's recorded pattern (the caller already ran it)."""
    import copy

    def fp64_in(pattern):
        # torch fp64 on the GPU when there is one (native im2col + dgemm for double convs:
        # MIOpen is fp32/16 only) — the same fp64 reference, minutes faster for ATF/R101
        d64 = "cuda" if torch.cuda.is_available() else "cpu"
        o64 = copy.deepcopy(o).double().to(d64)
        for p in o64.parameters():
            p.grad = None
        b64 = tuple((t.double() if t.is_floating_point() else t).to(d64) for t in cpu_batch)
        run_in_pattern(o64, pattern, lambda: run(o64, b64).backward())
        return {k: p.grad.detach().cpu() if p.grad is not None else None
                for k, p in o64.named_parameters()}

    og = copy.deepcopy(o).cuda()
    for p in og.parameters():
        p.grad = None
    gb = tuple(t.cuda() for t in cpu_batch)
    own_gpu = record_pattern(og, lambda: run(og, gb).backward())
    refs = {"device": fp64_in(device_forced(taps, n_rows)), "cpu32": fp64_in(own32),
            "gpu32": fp64_in(own_gpu)}
    runs = {"device": dict(m.named_parameters()), "cpu32": dict(o.named_parameters()),
            "gpu32": dict(og.named_parameters())}
    errs = {}
    for k, p in o.named_parameters():
        if not p.requires_grad or p.grad is None:
            continue
        e = []
        for name in ("device", "cpu32", "gpu32"):
            ref = refs[name][k].double()
            got = runs[name][k].grad.detach().double().cpu()
            e.append(float((got - ref).norm()) / max(float(ref.norm()), 1e-30))
        errs[k] = tuple(e)
    print({k: tuple(f"{x:.1e}" for x in v) for k, v in errs.items()})
    floor = float(os.environ.get("TLOD_GRAD_FLOOR", floor))  # diagnostics: a tighter floor
    bad = {k: v for k, v in errs.items() if v[0] > max(factor * max(v[1], v[2]), floor)}
    ratios = sorted(v[0] / max(v[1], v[2], 1e-12) for v in errs.values())
    worst = ratios[-1]
    print("device error: max", f"{max(v[0] for v in errs.values()):.2e}",
          "| device / max(cpu32, gpu32): median", round(ratios[len(ratios) // 2], 2),
          "max", round(worst, 2))
    assert not bad, {"violations": bad, "worst_ratio": worst}
    return errs


# ---------------------------------------------------------------- proposal sets
def box_iou(a, b):
    """(n,4) x (m,4) IoU, +1 pixel convention."""
    a, b = a.astype(np.float64), b.astype(np.float64)
    iw = np.minimum(a[:, None, 2], b[None, :, 2]) - np.maximum(a[:, None, 0], b[None, :, 0]) + 1
    ih = np.minimum(a[:, None, 3], b[None, :, 3]) - np.maximum(a[:, None, 1], b[None, :, 1]) + 1
    inter = np.clip(iw, 0, None) * np.clip(ih, 0, None)
    aa = (a[:, 2] - a[:, 0] + 1) * (a[:, 3] - a[:, 1] + 1)
    ab = (b[:, 2] - b[:, 0] + 1) * (b[:, 3] - b[:, 1] + 1)
    return inter / (aa[:, None] + ab[None, :] - inter)


def assert_proposal_sets_match(dev_rois, ref_rois, key):
    """a proposal layer's output on each side's own RPN outputs.  Near-tied
    random-init scores can reorder the sort and move the top-N boundary, so the proposals
    are compared as sets: >= 99.5% of each side's boxes have an IoU >= 0.999 partner on the
    other side, and the counts agree within 0.5%."""
    d = np.asarray(dev_rois).reshape(-1, 5)
    r = np.asarray(ref_rois).reshape(-1, 5)
    d = d[(d[:, 3] > d[:, 1]) | (d[:, 4] > d[:, 2])]  # drop the zero padding rows
    r = r[(r[:, 3] > r[:, 1]) | (r[:, 4] > r[:, 2])]
    assert len(r) > 0, key
    assert abs(len(d) - len(r)) <= max(2, len(r) // 200), (key, len(d), len(r))
    iou = box_iou(d[:, 1:], r[:, 1:])
    for side, best in (("device", iou.max(1)), ("oracle", iou.max(0))):
        frac = float((best >= 0.999).mean())
        assert frac >= 0.995, (key, side, frac)
