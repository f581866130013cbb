"""Microbenchmark: RoIAlignAvg 7x7 backward on the DAF step's shape (2 images, base feature
512 x 37 x 75, 256 source + 300 target RoIs of realistic sizes): the sorted-tap gather
(default, no atomics), TLOD_ROI_BWD_GATHER=0 the global-atomic NHWC kernel."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
from tlod import _lib  # noqa: E402


def main():
    dev = "cuda"
    B, C, H, W = 2, 512, 37, 75
    rng = np.random.default_rng(0)
    rois = []
    for b, n in ((0, 256), (1, 300)):
        x1 = rng.uniform(0, W * 16 - 64, n)
        y1 = rng.uniform(0, H * 16 - 64, n)
        w = rng.uniform(32, 600, n)
        h = rng.uniform(32, 400, n)
        rois.append(np.stack([np.full(n, b), x1, y1, np.minimum(x1 + w, W * 16 - 1),
                              np.minimum(y1 + h, H * 16 - 1)], 1))
    r = torch.from_numpy(np.concatenate(rois).astype(np.float32)).to(dev)
    R = r.shape[0]
    top = torch.randn(R, C, 7, 7, device=dev)
    grad = torch.zeros(B, C, H, W, device=dev)
    L = _lib.lib()
    wsb = max(L.tlod_roi_align_avg_bwd_gather_workspace_bytes(B, C, H, W, R, 7, 7),
              L.tlod_roi_align_avg_bwd_workspace_bytes(B, C, H, W))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def run():
        _lib.check(L.tlod_roi_align_avg_bwd_f32(_lib.ptr(top), B, C, H, W, _lib.ptr(r), R, 7, 7,
                                                1.0 / 16, _lib.ptr(grad), _lib.ptr(ws), ws.numel(),
                                                _lib.stream_of(top)), "roi_align_avg_bwd")
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    kind = "atomic" if os.environ.get("TLOD_ROI_BWD_GATHER") == "0" else "gather"
    print(json.dumps({"kernel": kind, "roi_align_avg_bwd_us": round(us, 1),
                      "R": R, "C": C, "map": [H, W]}))


if __name__ == "__main__":
    main()
