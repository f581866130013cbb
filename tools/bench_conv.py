"""Microbenchmark: VGG16 conv3_3 forward / dgrad / wgrad at batch 2 x 600 x 1000
(conv3 map 150 x 250, 256 -> 256, 3x3) — the north-star kernel (176.9 GFLOP
for the backward).  Times libtlod against torch (MIOpen) fp32 on the same data."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from tlod import conv as tc  # noqa: E402


def timeit(fn, iters, warmup=3):
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
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--H", type=int, default=150)
    ap.add_argument("--W", type=int, default=250)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch", action="store_true", help="also time MIOpen fp32")
    ap.add_argument("--math", default="f32", choices=tc.MATHS)
    a = ap.parse_args()
    dev = "cuda"
    N, C, H, W = a.N, a.C, a.H, a.W
    x = torch.randn(N, C, H, W, device=dev)
    w = torch.randn(C, C, 3, 3, device=dev) * (2.0 / (9 * C)) ** 0.5
    b = torch.zeros(C, device=dev)
    g = torch.randn(N, C, H, W, device=dev)
    flop = 2.0 * N * H * W * C * C * 9
    m = a.math
    wk = tc.pack_fwd(w) if m == "f32" else tc.pack_bs(w, False)
    wd = tc.pack_dgrad(w) if m == "f32" else tc.pack_bs(w, True)
    out = {"math": m}
    out["fwd_ms"] = timeit(lambda: tc.conv_fwd(x, w, b, True, wk=wk, math=m), a.iters)
    out["dgrad_ms"] = timeit(lambda: tc.conv_dgrad(g, w, wd=wd, math=m), a.iters)
    out["wgrad_ms"] = timeit(lambda: tc.conv_wgrad(g, x, 3, math=m), a.iters)
    if m != "f32":
        out["wgrad_f32_ms"] = timeit(lambda: tc.conv_wgrad(g, x, 3, math="f32"), a.iters)
    # the backward as the training step issues it: dgrad on the current stream, wgrad on a
    # side stream (independent: dgrad reads dY and W, wgrad dY and X), wall clock of the pair
    side = torch.cuda.Stream()
    dw = torch.empty_like(w)

    def pair():
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            tc.conv_wgrad(g, x, 3, out=dw, math=m)
        tc.conv_dgrad(g, w, wd=wd, math=m)
        torch.cuda.current_stream().wait_stream(side)
    out["bwd_pair_ms"] = timeit(pair, a.iters)
    # the same with dgrad on a high-priority stream: the dispatcher places every dgrad
    # workgroup before any wgrad one, wgrad filling dgrad's last partial round
    hi = torch.cuda.Stream(priority=-1)

    def pair_prio():
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(hi):
            hi.wait_event(ev)
            tc.conv_dgrad(g, w, wd=wd, math=m)
        with torch.cuda.stream(side):
            side.wait_event(ev)
            tc.conv_wgrad(g, x, 3, out=dw, math=m)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.current_stream().wait_stream(hi)
    out["bwd_pair_prio_ms"] = timeit(pair_prio, a.iters)
    for k in ("fwd", "dgrad", "wgrad"):
        out[k + "_tflops"] = flop / (out[k + "_ms"] * 1e-3) / 1e12
    bwd = out["dgrad_ms"] + out["wgrad_ms"]
    out["bwd_gflop"] = 2 * flop / 1e9
    out["bwd_tflops"] = 2 * flop / (bwd * 1e-3) / 1e12
    out["bwd_pair_tflops"] = 2 * flop / (out["bwd_pair_ms"] * 1e-3) / 1e12
    out["bwd_frac_f32_mfma_peak"] = out["bwd_tflops"] / 157.3
    if m != "f32":  # f32-equivalent peak of the split products
        out["bwd_frac_split_peak"] = out["bwd_tflops"] / (2516.6 / int(m[-1]))
        out["bwd_pair_frac_split_peak"] = out["bwd_pair_tflops"] / (2516.6 / int(m[-1]))
    if a.torch:
        xr = x.clone().requires_grad_(True)
        wr = w.clone().requires_grad_(True)
        out["miopen_fwd_ms"] = timeit(lambda: F.conv2d(x, w, b, padding=1), a.iters)

        def tb():
            torch.ops.aten.convolution_backward(g, x, w, [C], [1, 1], [1, 1], [1, 1], False,
                                                [0, 0], 1, [True, True, False])
        out["miopen_bwd_ms"] = timeit(tb, a.iters)
        out["miopen_bwd_tflops"] = 2 * flop / (out["miopen_bwd_ms"] * 1e-3) / 1e12
        del xr, wr
    print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
