"""Host side of the device input blob (csrc/blob.hip, tlod_image_blob_u8).

The kernel does the per-pixel work (BGR, mean subtraction, bilinear resize, crop / pad,
CHW); this module builds its small tables exactly as the reference's libraries do:

  * ``pixel_lut``: numpy's ``im.astype(np.float32); im -= PIXEL_MEANS`` (float64 means,
    lib/model/utils/blob.py:38-39) rounds ``v - mean`` once from double — tabulated for
    the 256 byte values of each channel;
  * ``linear_taps``: cv::resize INTER_LINEAR's per-column / per-row source index and
    weights for a scale factor given as fx (cv2.resize(im, None, None, fx=s, fy=s),
    blob.py:48-49): ``scale = 1/fx`` in double, ``f = float((d + 0.5) * scale - 0.5)``,
    ``s = floor(f)``, ``f -= s`` in float, clamped to weight 0 past either border;
  * ``resized_size``: cv::resize's output size, ``saturate_cast<int>(n * fx)`` (round half
    to even).
cv2 is not installed here (nor on the GPU box), so these restate OpenCV's published
INTER_LINEAR float path; the oracle (oracle/blob.py) restates it independently for the
parity tests ("parity unpinned" against cv2 itself: its SIMD build may fuse the vertical
multiply-add, a <= 1-ulp difference, and at an exact 2x downscale it switches to INTER_AREA,
which averages the same four pixels in another order).
"""
import numpy as np
import torch

from .. import _lib

TAP = np.dtype([("i0", np.int32), ("i1", np.int32), ("w0", np.float32), ("w1", np.float32)])


def pixel_lut(pixel_means):
    """3 x 256 float32: lut[c, v] = float32(float64(v) - pixel_means[c]) (BGR order)."""
    m = np.asarray(pixel_means, dtype=np.float64).reshape(3)
    v = np.arange(256, dtype=np.float64)
    return (v[None, :] - m[:, None]).astype(np.float32)


def resized_size(n, fx):
    return int(np.rint(n * float(fx)))


def linear_taps(src_len, dst_len, fx, flip=False):
    """cv::resize INTER_LINEAR taps of one axis (TAP records); flip mirrors the source
    index (the image was flipped before resizing, minibatch.py:75-76)."""
    scale = 1.0 / float(fx)
    d = np.arange(dst_len, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= src_len - 1
    f[hi], s[hi] = 0.0, src_len - 1
    t = np.empty(dst_len, TAP)
    i0, i1 = s, np.minimum(s + 1, src_len - 1)
    if flip:
        i0, i1 = src_len - 1 - i0, src_len - 1 - i1
    t["i0"], t["i1"] = i0, i1
    t["w0"] = (np.float32(1.0) - f).astype(np.float32)
    t["w1"] = f
    assert int(t["i0"].min()) >= 0 and int(t["i1"].max()) < src_len
    return t


def _dev(arr, device):
    """Pinned host copy -> device (non-blocking: the caller's stream orders it)."""
    host = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1)).pin_memory()
    return host.to(device, non_blocking=True)


def image_blob(src_u8, im_scale, pixel_means, flip=False, crop=(0, 0), keep_hw=None,
               out_hw=None):
    """One image -> its (3, Ho, Wo) float32 blob on the device.

    src_u8: (H, W, 3) uint8 RGB tensor on the device (or a numpy array, uploaded here);
    im_scale: cv2 fx = fy; crop (y0, x0) and keep_hw (Hd, Wd): the region of the resized
    image that is kept (default: everything from the offset on); out_hw: (Ho, Wo) of the
    zero-padded output (default keep_hw).  Returns (blob, (Hr, Wr)), Hr x Wr the resized
    size."""
    if isinstance(src_u8, np.ndarray):
        src_u8 = _dev(src_u8, torch.device("cuda", torch.cuda.current_device())).view(
            src_u8.shape)
    _lib.require_cuda(src_u8)
    assert src_u8.dtype == torch.uint8 and src_u8.dim() == 3 and src_u8.shape[2] == 3
    src_u8 = src_u8.contiguous()
    H, W = int(src_u8.shape[0]), int(src_u8.shape[1])
    Hr, Wr = resized_size(H, im_scale), resized_size(W, im_scale)
    y0, x0 = int(crop[0]), int(crop[1])
    Hd, Wd = (Hr - y0, Wr - x0) if keep_hw is None else (int(keep_hw[0]), int(keep_hw[1]))
    Ho, Wo = (Hd, Wd) if out_hw is None else (int(out_hw[0]), int(out_hw[1]))
    Hd, Wd = min(Hd, Ho), min(Wd, Wo)
    if y0 + Hd > Hr or x0 + Wd > Wr:
        raise ValueError(f"kept region {Hd}x{Wd}+{y0}+{x0} outside the resized {Hr}x{Wr}")
    dev = src_u8.device
    lut = _dev(pixel_lut(pixel_means), dev)
    xt = _dev(linear_taps(W, Wr, im_scale, flip), dev)
    yt = _dev(linear_taps(H, Hr, im_scale), dev)
    out = torch.empty((3, Ho, Wo), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().tlod_image_blob_u8(
        _lib.ptr(src_u8), H, W, _lib.ptr(lut), _lib.ptr(xt), _lib.ptr(yt), Hr, Wr, y0, x0, Hd,
        Wd, Ho, Wo, _lib.ptr(out), _lib.stream_of(src_u8)), "image_blob")
    return out, (Hr, Wr)
