"""Oracle: RoIAlign / RoIAlignAvg / RoIPool forward+backward, CUDA-kernel semantics.

Test infrastructure only (see oracle/__init__.py).  Type promotion follows the CUDA
source literally: expressions with a ``1.`` literal are double, everything else float.
"""
import numpy as np

f32 = np.float32
f64 = np.float64


def _align_geometry(rois, ah, aw, scale, H, W):
    """Per-(roi, ph, pw) sample geometry of ROIAlignForward/Backward
    (lib/model/roi_align/src/roi_align_kernel.cu:30-53 and :104-127)."""
    rois = rois.astype(np.float32)
    s = f32(scale)
    bidx = rois[:, 0].astype(np.int64)          # int img_start = roi_batch_ind * C*H*W
    sw = rois[:, 1] * s
    sh = rois[:, 2] * s
    ew = rois[:, 3] * s
    eh = rois[:, 4] * s
    # fmaxf(end - start + 1., 0.): float diff, +1 in double, rounded to float by fmaxf
    rw = np.maximum(((ew - sw).astype(f64) + 1.0).astype(f32), f32(0))
    rh = np.maximum(((eh - sh).astype(f64) + 1.0).astype(f32), f32(0))
    bh = (rh.astype(f64) / (ah - 1.0)).astype(f32)   # float / double -> stored as float
    bw = (rw.astype(f64) / (aw - 1.0)).astype(f32)
    ph = np.arange(ah, dtype=np.float32)
    pw = np.arange(aw, dtype=np.float32)
    h = (ph[None, :] * bh[:, None]).astype(f32) + sh[:, None]   # (R, ah) float ops
    w = (pw[None, :] * bw[:, None]).astype(f32) + sw[:, None]   # (R, aw)
    hs = np.minimum(np.floor(h), f32(H - 2)).astype(np.int64)  # fminf(floor(h), H-2)
    ws = np.minimum(np.floor(w), f32(W - 2)).astype(np.int64)
    hr = (h - hs.astype(f32)).astype(f32)
    wr = (w - ws.astype(f32)).astype(f32)
    hvalid = ~((h < 0) | (h >= H))
    wvalid = ~((w < 0) | (w >= W))
    return bidx, hs, ws, hr, wr, hvalid, wvalid


def roi_align_fwd(feat, rois, ah, aw, scale):
    """ROIAlignForward (roi_align_kernel.cu:15-70): (B,C,H,W),(R,5) -> (R,C,ah,aw) float32."""
    feat = np.ascontiguousarray(feat, dtype=np.float32)
    B, C, H, W = feat.shape
    R = rois.shape[0]
    bidx, hs, ws, hr, wr, hv, wv = _align_geometry(rois, ah, aw, scale, H, W)
    out = np.zeros((R, C, ah, aw), np.float32)
    for r in range(R):
        f = feat[bidx[r]]
        y = np.clip(hs[r], 0, H - 2)[:, None]
        x = np.clip(ws[r], 0, W - 2)[None, :]
        h_r = hr[r][:, None]                       # float32 (ah,1)
        w_r = wr[r][None, :]                       # float32 (1,aw)
        ul, ur = f[:, y, x], f[:, y, x + 1]        # (C, ah, aw)
        dl, dr = f[:, y + 1, x], f[:, y + 1, x + 1]
        t1 = (ul.astype(f64) * (1.0 - h_r.astype(f64))) * (1.0 - w_r.astype(f64))
        t2 = (ur.astype(f64) * (1.0 - h_r.astype(f64))) * w_r.astype(f64)
        t3 = (dl * h_r).astype(f32).astype(f64) * (1.0 - w_r.astype(f64))
        t4 = ((dr * h_r).astype(f32) * w_r).astype(f32).astype(f64)
        v = (((t1 + t2) + t3) + t4).astype(f32)
        valid = (hv[r][:, None] & wv[r][None, :])[None]
        out[r] = np.where(valid, v, f32(0))
    return out


def roi_align_bwd(top_grad, rois, B, C, H, W, scale):
    """ROIAlignBackward (roi_align_kernel.cu:94-143): 4 atomicAdds per sample.

    Accumulated in float64 (the reference's atomic order is nondeterministic); the
    per-tap contribution is rounded to float exactly as the atomicAdd argument is."""
    R, _, ah, aw = top_grad.shape
    bidx, hs, ws, hr, wr, hv, wv = _align_geometry(rois, ah, aw, scale, H, W)
    acc = np.zeros(B * C * H * W, np.float64)
    cidx = np.arange(C)[:, None, None]
    idx_chunks, val_chunks = [], []

    def flush():
        if idx_chunks:
            acc[:] += np.bincount(np.concatenate(idx_chunks), np.concatenate(val_chunks),
                                  minlength=acc.size)
            idx_chunks.clear()
            val_chunks.clear()

    for r in range(R):
        valid = (hv[r][:, None] & wv[r][None, :])
        if not valid.any():
            continue
        y = np.clip(hs[r], 0, H - 2)[:, None] + np.zeros((1, aw), np.int64)
        x = np.clip(ws[r], 0, W - 2)[None, :] + np.zeros((ah, 1), np.int64)
        h_r = np.broadcast_to(hr[r][:, None], (ah, aw)).astype(f32)
        w_r = np.broadcast_to(wr[r][None, :], (ah, aw)).astype(f32)
        td = top_grad[r].astype(np.float32)              # (C, ah, aw)
        om = (f32(1) - w_r).astype(f32)                  # (1 - w_ratio): float
        c_ul = ((td.astype(f64) * (1.0 - h_r.astype(f64))) * om.astype(f64)).astype(f32)
        c_ur = ((td.astype(f64) * (1.0 - h_r.astype(f64))) * w_r.astype(f64)).astype(f32)
        c_dl = ((td * h_r).astype(f32) * om).astype(f32)
        c_dr = ((td * h_r).astype(f32) * w_r).astype(f32)
        m = np.broadcast_to(valid[None], td.shape)
        base = (bidx[r] * C + np.broadcast_to(cidx, td.shape)[m]) * H
        yy = np.broadcast_to(y[None], td.shape)[m]
        xx = np.broadcast_to(x[None], td.shape)[m]
        ul = (base + yy) * W + xx
        dl = (base + yy + 1) * W + xx
        idx_chunks += [ul, ul + 1, dl, dl + 1]
        val_chunks += [c_ul[m], c_ur[m], c_dl[m], c_dr[m]]
        if len(idx_chunks) >= 128:
            flush()
    flush()
    acc = acc.reshape(B, C, H, W)
    return acc.astype(np.float32)


def avg_pool_2x2_s1(x):
    """torch avg_pool2d(kernel 2, stride 1) CUDA forward: ((((0+a)+b)+c)+d)/4 in float."""
    x = x.astype(np.float32)
    s = (x[..., :-1, :-1] + x[..., :-1, 1:]).astype(f32)
    s = (s + x[..., 1:, :-1]).astype(f32)
    s = (s + x[..., 1:, 1:]).astype(f32)
    return (s / f32(4)).astype(f32)


def avg_pool_2x2_s1_bwd(g):
    """torch avg_pool2d backward CUDA: grad_in[y][x] = sum_{py,px} g[py][px]/4, py outer."""
    g = g.astype(np.float32)
    oh, ow = g.shape[-2:]
    out = np.zeros(g.shape[:-2] + (oh + 1, ow + 1), np.float32)
    q = (g / f32(4)).astype(f32)
    for y in range(oh + 1):
        for x in range(ow + 1):
            acc = np.zeros(g.shape[:-2], np.float32)
            for py in range(max(0, y - 1), min(y, oh - 1) + 1):
                for px in range(max(0, x - 1), min(x, ow - 1) + 1):
                    acc = (acc + q[..., py, px]).astype(f32)
            out[..., y, x] = acc
    return out


def roi_align_avg_fwd(feat, rois, pooled_h, pooled_w, scale):
    """RoIAlignAvg (lib/model/roi_align/modules/roi_align.py:18-29): align (p+1)^2 then avg 2x2/s1."""
    return avg_pool_2x2_s1(roi_align_fwd(feat, rois, pooled_h + 1, pooled_w + 1, scale))


def roi_align_avg_bwd(top_grad, rois, B, C, H, W, scale):
    return roi_align_bwd(avg_pool_2x2_s1_bwd(top_grad), rois, B, C, H, W, scale)


# ------------------------------------------------------------------ RoIPool
def _c_round(x):
    """C round() of a float promoted to double: half away from zero."""
    x = x.astype(f64)
    return (np.sign(x) * np.floor(np.abs(x) + 0.5)).astype(np.int64)


def _pool_rois(rois, scale):
    rois = rois.astype(np.float32)
    s = f32(scale)
    b = rois[:, 0].astype(np.int64)
    sw = _c_round(rois[:, 1] * s)
    sh = _c_round(rois[:, 2] * s)
    ew = _c_round(rois[:, 3] * s)
    eh = _c_round(rois[:, 4] * s)
    rw = np.maximum(ew - sw + 1, 1)
    rh = np.maximum(eh - sh + 1, 1)
    return b, sw, sh, ew, eh, rw, rh


def roi_pool_fwd(feat, rois, ph_n, pw_n, scale):
    """ROIPoolForward (lib/model/roi_pooling/src/roi_pooling_kernel.cu:24-93).

    Returns (out (R,C,ph,pw) float32, argmax int32 flat index into feat, -1 if empty)."""
    feat = np.ascontiguousarray(feat, dtype=np.float32)
    B, C, H, W = feat.shape
    R = rois.shape[0]
    b, sw, sh, ew, eh, rw, rh = _pool_rois(rois, scale)
    out = np.zeros((R, C, ph_n, pw_n), np.float32)
    arg = np.full((R, C, ph_n, pw_n), -1, np.int32)
    for r in range(R):
        bsh = f32(rh[r]) / f32(ph_n)
        bsw = f32(rw[r]) / f32(pw_n)
        for ph in range(ph_n):
            hs = int(np.floor(f32(ph) * bsh))
            he = int(np.ceil(f32(ph + 1) * bsh))
            hs = min(max(hs + sh[r], 0), H)
            he = min(max(he + sh[r], 0), H)
            for pw in range(pw_n):
                ws = int(np.floor(f32(pw) * bsw))
                we = int(np.ceil(f32(pw + 1) * bsw))
                ws = min(max(ws + sw[r], 0), W)
                we = min(max(we + sw[r], 0), W)
                if he <= hs or we <= ws:
                    continue  # maxval 0, argmax -1
                win = feat[b[r], :, hs:he, ws:we].reshape(C, -1)
                k = np.argmax(win, axis=1)                 # first max == strict '>' scan
                out[r, :, ph, pw] = win[np.arange(C), k]
                wh = we - ws
                hh = hs + k // wh
                ww = ws + k % wh
                arg[r, :, ph, pw] = ((b[r] * C + np.arange(C)) * H + hh) * W + ww
    return out, arg


def roi_pool_bwd(top_grad, argmax, rois, B, C, H, W, scale):
    """ROIPoolBackward (roi_pooling_kernel.cu:128-203), a gather over RoIs per input element.

    Restated as the equivalent scatter: contribution (r,c,ph,pw) reaches input index
    argmax iff argmax >= 0, the element lies inside the (unclipped, inclusive) RoI
    (:160-164) and (ph,pw) lies in the feasible bin range computed at :175-186."""
    R, _, ph_n, pw_n = top_grad.shape
    b, sw, sh, ew, eh, rw, rh = _pool_rois(rois, scale)
    acc = np.zeros(B * C * H * W, np.float64)
    for r in range(R):
        a = argmax[r].reshape(-1).astype(np.int64)
        g = top_grad[r].reshape(-1).astype(np.float64)
        ok = a >= 0
        idx = np.where(ok, a, 0)
        w = idx % W
        h = (idx // W) % H
        n = idx // (W * H * C)
        ok &= n == b[r]
        ok &= (w >= sw[r]) & (w <= ew[r]) & (h >= sh[r]) & (h <= eh[r])
        bsh = f32(rh[r]) / f32(ph_n)
        bsw = f32(rw[r]) / f32(pw_n)
        phs = np.floor(((h - sh[r]).astype(f32) / bsh).astype(f32)).astype(np.int64)
        phe = np.ceil(((h - sh[r] + 1).astype(f32) / bsh).astype(f32)).astype(np.int64)
        pws = np.floor(((w - sw[r]).astype(f32) / bsw).astype(f32)).astype(np.int64)
        pwe = np.ceil(((w - sw[r] + 1).astype(f32) / bsw).astype(f32)).astype(np.int64)
        phs, phe = np.clip(phs, 0, ph_n), np.clip(phe, 0, ph_n)
        pws, pwe = np.clip(pws, 0, pw_n), np.clip(pwe, 0, pw_n)
        ph = np.tile(np.repeat(np.arange(ph_n), pw_n), C)
        pw = np.tile(np.arange(pw_n), C * ph_n)
        ok &= (ph >= phs) & (ph < phe) & (pw >= pws) & (pw < pwe)
        np.add.at(acc, idx[ok], g[ok])
    return acc.astype(np.float32).reshape(B, C, H, W)


# ------------------------------------------------------------------ float64 reference
# The same function in float64 arithmetic: the sample geometry (bin positions, integer
# taps, fractional weights) is the kernels' float32 geometry — it defines which function
# is computed — and every value / gradient operation after it is double.  Used as the
# "exact" side of the gradient accuracy bars (tests/helpers.grad_error_bar).
def roi_align_avg_fwd64(feat, rois, pooled_h, pooled_w, scale):
    feat = np.asarray(feat, dtype=f64)
    B, C, H, W = feat.shape
    ah, aw = pooled_h + 1, pooled_w + 1
    bidx, hs, ws, hr, wr, hv, wv = _align_geometry(rois, ah, aw, scale, H, W)
    out = np.zeros((rois.shape[0], C, ah, aw), f64)
    for r in range(rois.shape[0]):
        f = feat[bidx[r]]
        y = np.clip(hs[r], 0, H - 2)[:, None]
        x = np.clip(ws[r], 0, W - 2)[None, :]
        h_r, w_r = hr[r][:, None].astype(f64), wr[r][None, :].astype(f64)
        v = (f[:, y, x] * (1 - h_r) * (1 - w_r) + f[:, y, x + 1] * (1 - h_r) * w_r
             + f[:, y + 1, x] * h_r * (1 - w_r) + f[:, y + 1, x + 1] * h_r * w_r)
        out[r] = np.where((hv[r][:, None] & wv[r][None, :])[None], v, 0.0)
    return (out[..., :-1, :-1] + out[..., :-1, 1:] + out[..., 1:, :-1] + out[..., 1:, 1:]) / 4.0


def roi_align_avg_bwd64(top_grad, rois, B, C, H, W, scale):
    g = np.asarray(top_grad, dtype=f64) / 4.0
    R, _, ph, pw = g.shape
    ah, aw = ph + 1, pw + 1
    ga = np.zeros((R, C, ah, aw), f64)
    ga[..., :-1, :-1] += g
    ga[..., :-1, 1:] += g
    ga[..., 1:, :-1] += g
    ga[..., 1:, 1:] += g
    bidx, hs, ws, hr, wr, hv, wv = _align_geometry(rois, ah, aw, scale, H, W)
    acc = np.zeros((B, C, H, W), f64)
    for r in range(R):
        valid = (hv[r][:, None] & wv[r][None, :])[None]
        t = np.where(valid, ga[r], 0.0)
        y = np.clip(hs[r], 0, H - 2)
        x = np.clip(ws[r], 0, W - 2)
        h_r, w_r = hr[r][:, None].astype(f64), wr[r][None, :].astype(f64)
        for (dy, dx, wgt) in ((0, 0, (1 - h_r) * (1 - w_r)), (0, 1, (1 - h_r) * w_r),
                              (1, 0, h_r * (1 - w_r)), (1, 1, h_r * w_r)):
            yy = np.broadcast_to((y + dy)[:, None], (ah, aw)).reshape(-1)
            xx = np.broadcast_to((x + dx)[None, :], (ah, aw)).reshape(-1)
            np.add.at(acc[bidx[r]], (slice(None), yy, xx), (t * wgt).reshape(C, -1))
    return acc
