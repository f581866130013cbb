"""Per-chunk vs per-tile cost of the split-bf16 3x3 conv kernels: time fwd (the
warp-specialized kernel for Cin >= 128), dgrad and wgrad at a fixed map and Cout while Cin
grows, so that T(Cin) = fixed + Cin x marginal separates the K loop from the per-tile
prologue / epilogue / tail.  usage: python tools/conv_scan.py [--H 150 --W 250 --Cout 256]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))

import torch  # noqa: E402

from tlod import conv as tc  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=2)
    ap.add_argument("--H", type=int, default=150)
    ap.add_argument("--W", type=int, default=250)
    ap.add_argument("--Cout", type=int, default=256)
    ap.add_argument("--cins", default="128,256,384,512")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N, H, W, Co = a.N, a.H, a.W, a.Cout
    rows = []
    for Ci in [int(c) for c in a.cins.split(",")]:
        x = torch.randn(N, Ci, H, W, device="cuda")
        w = torch.randn(Co, Ci, 3, 3, device="cuda") * (2.0 / (9 * Ci)) ** 0.5
        b = torch.zeros(Co, device="cuda")
        g = torch.randn(N, Co, H, W, device="cuda")
        wk = tc.pack_bs(w, False)
        wd = tc.pack_bs(w, True)
        flop = 2.0 * N * H * W * Co * Ci * 9
        r = {"Cin": Ci, "Cout": Co, "H": H, "W": W}
        r["fwd_ms"] = timeit(lambda: tc.conv_fwd(x, w, b, True, wk=wk, math="bf16x6"), a.iters)
        r["wgrad_ms"] = timeit(lambda: tc.conv_wgrad(g, x, 3, math="bf16x6"), a.iters)
        if Ci == Co:
            r["dgrad_ms"] = timeit(lambda: tc.conv_dgrad(g, w, wd=wd, math="bf16x6"), a.iters)
        for k in ("fwd", "wgrad", "dgrad"):
            if k + "_ms" in r:
                r[k + "_tf"] = round(flop / (r[k + "_ms"] * 1e-3) / 1e12, 1)
                r[k + "_ms"] = round(r[k + "_ms"], 4)
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w, g, wk, wd
    if len(rows) >= 2:
        for k in ("fwd", "wgrad"):
            c0, c1 = rows[0]["Cin"], rows[-1]["Cin"]
            t0, t1 = rows[0][k + "_ms"], rows[-1][k + "_ms"]
            marg = (t1 - t0) / (c1 - c0)
            fixed = t0 - marg * c0
            mflop = 2.0 * N * H * W * Co * 9  # per input channel
            print(json.dumps({"kind": k, "marginal_ms_per_cin": round(marg, 6),
                              "fixed_ms": round(fixed, 4),
                              "marginal_tf": round(mflop / (marg * 1e-3) / 1e12, 1)}))


if __name__ == "__main__":
    main()
