"""Diagnostic: per-segment cycle sums of the warp-specialized conv loop (stamp build).
usage: TLOD_LIB=build_variants/stamps/libtlod.so TLOD_CONV_WS=2 python ws_stamps.py"""
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
w = torch.randn(C, C, 3, 3, device="cuda") * (2.0 / (9 * C)) ** 0.5
b = torch.zeros(C, device="cuda")
wk = tc.pack_bs(w, False)
for _ in range(30):
    tc.conv_fwd(x, w, b, True, wk=wk, math="bf16x6")
torch.cuda.synchronize()
buf = np.zeros(256 * 12 * 10 + 512, np.uint64)
f = _lib.lib().tlod_debug_ws_stamps
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
a = buf[:256 * 12 * 10].reshape(256, 12, 10).astype(np.float64)
names = ["work (k-steps | staging)", "wait F1 (flags: all waits)", "wait F2", "wait F3", "wait F4",
         "wait F5", "wait F6", "wait F7", "first barrier", "epilogue"]
for role, sl in (("MFMA waves", slice(0, 8)), ("producer waves", slice(8, 12))):
    v = a[:, sl, :]
    tot = v.sum(-1)
    print(f"{role}: total cycles per wave median {np.median(tot):.0f}")
    for k, nm in enumerate(names):
        print(f"   {nm:34s} median {np.median(v[:, :, k]):10.0f}  frac {np.median(v[:, :, k] / tot):.3f}")
clk = buf[256 * 12 * 10:].reshape(256, 2).astype(np.float64)
print("block-0 wave-0 span: cycles %.0f, realtime %.0f us, clock %.3f GHz (median over blocks %.3f)" % (
    clk[0, 0], clk[0, 1] / 100.0, clk[0, 0] / clk[0, 1] / 10.0, np.median(clk[:, 0] / clk[:, 1] / 10.0)))

# per-block timeline of the last launch (s_memrealtime, 100 MHz): rounds and tail
f2 = _lib.lib().tlod_debug_ws_timeline
f2.argtypes = [ctypes.c_void_p]
tl = np.zeros(8192 * 2, np.uint64)
torch.cuda.synchronize()
tl[:] = 0
assert f2(tl.ctypes.data) == 0
tl = tl.reshape(8192, 2).astype(np.float64)
nb = int((tl[:, 1] > 0).sum())
t = tl[:nb] - tl[:nb, 0].min()
dur = (t[:, 1] - t[:, 0]) / 100.0
print("blocks %d, kernel span %.1f us, block duration us: min %.1f median %.1f max %.1f" % (
    nb, t[:, 1].max() / 100.0, dur.min(), np.median(dur), dur.max()))
st = np.sort(t[:, 0]) / 100.0
print("block start times (us) at quantiles 0, .25, .5, .75, 1:", np.round(np.quantile(st, [0, .25, .5, .75, 1]), 1))
busy = np.zeros(int(t[:, 1].max() / 100.0) + 1)
for s0, e0 in t / 100.0:
    busy[int(s0):int(e0)] += 1
print("resident blocks per 10-us bin:", [int(busy[i:i + 10].mean()) for i in range(0, len(busy), 10)])
