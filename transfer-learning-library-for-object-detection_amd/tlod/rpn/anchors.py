"""Reference anchor windows (lib/model/rpn/generate_anchors.py:45-105), vectorised.

Windows are enumerated ratio-major then scale, around the base_size x base_size cell
(0, 0, 15, 15), widths/heights rounded half-to-even like ``np.round``.
"""
import numpy as np
import torch


def generate_anchors(base_size=16, ratios=(0.5, 1, 2), scales=(8, 16, 32)):
    ratios = np.asarray(ratios, dtype=np.float64).reshape(-1, 1)
    scales = np.asarray(scales, dtype=np.float64).reshape(1, -1)
    side = float(base_size)
    ctr = 0.5 * (side - 1.0)                       # centre of the (0,0,s-1,s-1) window
    ws = np.round(np.sqrt(side * side / ratios))   # (R,1) per-ratio width
    hs = np.round(ws * ratios)
    w = (ws * scales).reshape(-1)                  # ratio-major, scale-minor
    h = (hs * scales).reshape(-1)
    half_w, half_h = 0.5 * (w - 1.0), 0.5 * (h - 1.0)
    return np.stack([ctr - half_w, ctr - half_h, ctr + half_w, ctr + half_h], 1)


def base_anchor_tensor(scales, ratios, device=None):
    """(A,4) float32 tensor, as ``torch.from_numpy(generate_anchors(...)).float()``."""
    a = generate_anchors(scales=np.array(scales), ratios=np.array(ratios))
    return torch.from_numpy(a).float().to(device) if device is not None else torch.from_numpy(a).float()
