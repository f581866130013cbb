"""Diagnostic: per-segment cycle sums of the warp-specialized weight-gradient kernel (stamp
build: EXTRA_SRCS=wgrad_ws.hip tools/build_variants.sh wgstamps -DTLOD_WGWS_STAMPS=1).
usage: TLOD_LIB=build_variants/wgstamps/libtlod.so python tools/wgws_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "transfer-learning-library-for-object-detection_amd"))
from tlod import _lib, conv as tc  # noqa: E402

N, C, H, W = 2, int(os.environ.get("C", 256)), int(os.environ.get("H", 150)), int(os.environ.get("W", 250))
x = torch.randn(N, C, H, W, device="cuda")
g = torch.randn(N, C, H, W, device="cuda")
for _ in range(30):
    tc.conv_wgrad(g, x, 3, math="bf16x6")
torch.cuda.synchronize()
buf = np.zeros(256 * 12 * 4 + 512, np.uint64)
f = _lib.lib().tlod_debug_wgws_stamps
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
a = buf[:256 * 48].reshape(256, 12, 4).astype(np.float64)
for role, sl, names in (("MFMA waves", slice(0, 8), ["k-steps", "barrier waits", "epilogue", "first barrier"]),
                        ("producer waves", slice(8, 12), ["staging", "barrier waits", "load wait", "-"])):
    v = a[:, sl, :]
    tot = v.sum(-1)
    print(f"{role}: total cycles per wave median {np.median(tot):.0f}")
    for k, nm in enumerate(names):
        print(f"   {nm:20s} median {np.median(v[:, :, k]):10.0f}  frac {np.median(v[:, :, k] / np.maximum(tot, 1)):.3f}")
clk = buf[256 * 48:].reshape(256, 2).astype(np.float64)
print("block span median: cycles %.0f, %.1f us, clock %.3f GHz" % (
    np.median(clk[:, 0]), np.median(clk[:, 1]) / 100.0, np.median(clk[:, 0] / clk[:, 1] / 10.0)))
