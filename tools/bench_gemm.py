"""Microbenchmark: the head GEMMs (fc6 25088->4096, fc7 4096->4096 at R = 556 RoIs =
256 source + 300 target) forward / dgrad / wgrad: libtlod split-bf16 vs torch fp32."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.linear import gemm  # noqa: E402


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
R = 556
LAYERS = [("fc6", 25088, 4096), ("fc7", 4096, 4096)]
if "--r101" in sys.argv:  # the DAF-R101 RoI head's layer4 GEMMs: 428 RoIs x 16 bins (4 x 4)
    R = 6848
    LAYERS = [("l4_conv1", 2048, 512), ("l4_conv2", 4608, 512), ("l4_conv3", 512, 2048)]
if "--atf" in sys.argv:  # the ATF-R101 RoI head (config 5): 4512 RoIs x 16 bins through layer4
    R = int(os.environ.get("ATF_ROWS", 4512 * 16))
    LAYERS = [("l4b0_conv1", 1024, 512), ("l4_conv1", 2048, 512), ("l4_conv2", 4608, 512),
              ("l4_conv3", 512, 2048), ("l4_ds", 1024, 2048)]
if "--da" in sys.argv:  # the DAF instance-DA head (lib/DAF/DA.py:53-73) on the 556 RoIs
    LAYERS = [("ins_fc1", 4096, 1024), ("ins_fc2", 1024, 1024)]
NOTORCH = "--no-torch" in sys.argv
for name, I, O in LAYERS:
    x = torch.randn(R, I, device="cuda")
    w = torch.randn(O, I, device="cuda") * 0.01
    dy = torch.randn(R, O, device="cuda")
    f = 2.0 * R * I * O
    for kind, fn, tfn in (
            ("fwd", lambda: gemm(x, w, R, O, I, 1, 1), lambda: x @ w.t()),
            ("dgrad", lambda: gemm(dy, w, R, I, O, 1, 0), lambda: dy @ w),
            ("wgrad", lambda: gemm(dy, x, O, I, R, 0, 0), lambda: dy.t() @ x)):
        ms = timeit(fn)
        tms = float("nan") if NOTORCH else timeit(tfn)
        out[f"{name}_{kind}"] = {"ms": round(ms, 4), "tflops": round(f / ms / 1e9, 1),
                                 "torch_f32_ms": round(tms, 4),
                                 "torch_tflops": round(f / tms / 1e9, 1)}
print(json.dumps(out))
