"""Oracle: anchors, box transforms, IoU (test infrastructure only; see oracle/__init__.py).

All float work is float32 with one rounding per op, matching torch-CUDA elementwise
kernels (each op its own kernel, so no contraction happens in the reference either).
"""
import numpy as np

f32 = np.float32


# ---------------------------------------------------------------- anchors
def generate_anchors(base_size=16, ratios=(0.5, 1, 2), scales=(8, 16, 32)):
    """lib/model/rpn/generate_anchors.py:45-105 (float64 numpy, np.round = half-to-even).

    Returns (A, 4) float32 ordered ratio-major then scale, as ``np.vstack`` of
    ``_scale_enum`` over ``_ratio_enum`` rows (generate_anchors.py:52-54).
    """
    ratios = np.asarray(ratios, dtype=np.float64)
    scales = np.asarray(scales, dtype=np.float64)
    base = np.array([1, 1, base_size, base_size], dtype=np.float64) - 1

    def whctrs(a):  # generate_anchors.py:57-66
        w = a[2] - a[0] + 1
        h = a[3] - a[1] + 1
        return w, h, a[0] + 0.5 * (w - 1), a[1] + 0.5 * (h - 1)

    def mk(ws, hs, xc, yc):  # generate_anchors.py:68-81
        ws = ws[:, None]
        hs = hs[:, None]
        return np.hstack((xc - 0.5 * (ws - 1), yc - 0.5 * (hs - 1),
                          xc + 0.5 * (ws - 1), yc + 0.5 * (hs - 1)))

    w, h, xc, yc = whctrs(base)  # _ratio_enum :83-94
    size = w * h
    ws = np.round(np.sqrt(size / ratios))
    hs = np.round(ws * ratios)
    ratio_anchors = mk(ws, hs, xc, yc)
    out = []
    for i in range(ratio_anchors.shape[0]):  # _scale_enum :96-105
        w, h, xc, yc = whctrs(ratio_anchors[i])
        out.append(mk(w * scales, h * scales, xc, yc))
    return np.vstack(out).astype(np.float32)  # torch.from_numpy(...).float()


def shifted_anchors(base_anchors, feat_h, feat_w, feat_stride):
    """proposal_layer.py:80-93 / anchor_target_layer.py:66-79.

    all_anchors[(h*W + w)*A + a] = base[a] + (w*s, h*s, w*s, h*s), float32 add.
    """
    sx = (np.arange(feat_w) * feat_stride)
    sy = (np.arange(feat_h) * feat_stride)
    sx, sy = np.meshgrid(sx, sy)
    shifts = np.vstack((sx.ravel(), sy.ravel(), sx.ravel(), sy.ravel())).T.astype(np.float32)
    A = base_anchors.shape[0]
    K = shifts.shape[0]
    return (base_anchors.reshape(1, A, 4) + shifts.reshape(K, 1, 4)).reshape(K * A, 4).astype(np.float32)


# ---------------------------------------------------------------- transforms
def bbox_transform_inv(boxes, deltas):
    """bbox_transform.py:77-103 for one image: boxes (N,4), deltas (N,4) float32."""
    boxes = boxes.astype(np.float32)
    deltas = deltas.astype(np.float32)
    one, half = f32(1.0), f32(0.5)
    widths = boxes[:, 2] - boxes[:, 0] + one
    heights = boxes[:, 3] - boxes[:, 1] + one
    ctr_x = boxes[:, 0] + half * widths
    ctr_y = boxes[:, 1] + half * heights
    dx, dy, dw, dh = deltas[:, 0], deltas[:, 1], deltas[:, 2], deltas[:, 3]
    pcx = dx * widths + ctr_x
    pcy = dy * heights + ctr_y
    pw = np.exp(dw) * widths
    ph = np.exp(dh) * heights
    out = np.empty_like(deltas)
    out[:, 0] = pcx - half * pw
    out[:, 1] = pcy - half * ph
    out[:, 2] = pcx + half * pw
    out[:, 3] = pcy + half * ph
    return out


def clip_boxes(boxes, im_h, im_w):
    """bbox_transform.py:125-133: clamp x to [0, W-1], y to [0, H-1] (float32)."""
    b = boxes.copy()
    xm = f32(im_w) - f32(1)
    ym = f32(im_h) - f32(1)
    b[:, 0] = np.clip(b[:, 0], f32(0), xm)
    b[:, 1] = np.clip(b[:, 1], f32(0), ym)
    b[:, 2] = np.clip(b[:, 2], f32(0), xm)
    b[:, 3] = np.clip(b[:, 3], f32(0), ym)
    return b


def bbox_transform(ex, gt):
    """bbox_transform.py:36-75 (bbox_transform_batch) for one image: (N,4),(N,4) -> (N,4)."""
    ex = ex.astype(np.float32)
    gt = gt.astype(np.float32)
    one, half = f32(1.0), f32(0.5)
    ew = ex[:, 2] - ex[:, 0] + one
    eh = ex[:, 3] - ex[:, 1] + one
    ecx = ex[:, 0] + half * ew
    ecy = ex[:, 1] + half * eh
    gw = gt[:, 2] - gt[:, 0] + one
    gh = gt[:, 3] - gt[:, 1] + one
    gcx = gt[:, 0] + half * gw
    gcy = gt[:, 1] + half * gh
    return np.stack(((gcx - ecx) / ew, (gcy - ecy) / eh,
                     np.log(gw / ew), np.log(gh / eh)), 1).astype(np.float32)


# ---------------------------------------------------------------- IoU
def bbox_overlaps(anchors, gt):
    """bbox_transform.py:168-213 (bbox_overlaps_batch, anchors.dim()==2) for one image.

    anchors (N,4), gt (K,>=4) -> (N,K) float32, with the reference's masks:
    zero-area gt (w==1 & h==1) -> 0; zero-area anchor -> -1 (applied last).
    """
    a = anchors.astype(np.float32)
    g = gt[:, :4].astype(np.float32)
    one = f32(1)
    gx = g[:, 2] - g[:, 0] + one
    gy = g[:, 3] - g[:, 1] + one
    garea = gx * gy
    ax = a[:, 2] - a[:, 0] + one
    ay = a[:, 3] - a[:, 1] + one
    aarea = ax * ay
    gzero = (gx == 1) & (gy == 1)
    azero = (ax == 1) & (ay == 1)
    iw = np.minimum(a[:, None, 2], g[None, :, 2]) - np.maximum(a[:, None, 0], g[None, :, 0]) + one
    iw[iw < 0] = 0
    ih = np.minimum(a[:, None, 3], g[None, :, 3]) - np.maximum(a[:, None, 1], g[None, :, 1]) + one
    ih[ih < 0] = 0
    inter = iw * ih
    ua = aarea[:, None] + garea[None, :] - inter
    ov = (inter / ua).astype(np.float32)
    ov[:, gzero] = 0
    ov[azero, :] = -1
    return ov


def iou_pair_cuda(a, b):
    """devIoU (lib/model/nms/src/nms_cuda_kernel.cu:31-39), vectorised over b. float32."""
    one, zero = f32(1), f32(0)
    left = np.maximum(a[0], b[:, 0])
    right = np.minimum(a[2], b[:, 2])
    top = np.maximum(a[1], b[:, 1])
    bottom = np.minimum(a[3], b[:, 3])
    width = np.maximum(right - left + one, zero)
    height = np.maximum(bottom - top + one, zero)
    inter = width * height
    sa = (a[2] - a[0] + one) * (a[3] - a[1] + one)
    sb = (b[:, 2] - b[:, 0] + one) * (b[:, 3] - b[:, 1] + one)
    return inter / (sa + sb - inter)
