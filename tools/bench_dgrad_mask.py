"""Microbenchmark: the split-bf16 3x3 input gradient with and without the fused ReLU-mask
epilogue (tlod_conv_dgrad_bs_mask_f32) on the DAF-VGG16 step's shapes, beside the forward."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "transfer-learning-library-for-object-detection_amd"))
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


out = {}
for N, C, Co, H, W in [(2, 256, 256, 150, 300), (2, 512, 512, 75, 150), (2, 512, 512, 37, 75),
                       (2, 256, 256, 150, 250)]:
    x = torch.relu(torch.randn(N, C, H, W, device="cuda"))
    w = torch.randn(Co, C, 3, 3, device="cuda") * (2.0 / (9 * C)) ** 0.5
    b = torch.zeros(Co, device="cuda")
    g = torch.randn(N, Co, H, W, device="cuda")
    wk, wd = tc.pack_bs(w, False), tc.pack_bs(w, True)
    f = 2.0 * N * H * W * C * Co * 9
    r = {"fwd": timeit(lambda: tc.conv_fwd(x, w, b, True, wk=wk, math="bf16x6")),
         "dgrad": timeit(lambda: tc.conv_dgrad(g, w, wd=wd, math="bf16x6")),
         "dgrad_mask": timeit(lambda: tc.conv_dgrad(g, w, wd=wd, math="bf16x6", mask=x)),
         "wgrad": timeit(lambda: tc.conv_wgrad(g, x, 3, math="bf16x6"))}
    out[str((N, C, Co, H, W))] = {k: {"ms": round(v, 4), "tf": round(f / v / 1e9, 1)} for k, v in r.items()}
print(json.dumps(out))
