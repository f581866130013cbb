"""Which Python lines launch the torch-side (non-libtlod) GPU time of a training step:
torch.profiler over a few steps, the torch ops ranked by self device time with their input
shapes and the innermost tlod/ frame of their call stack.
usage: python tools/torch_prof.py [method] [net] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from tlod.detector.train import (SyntheticCityscapes, build_model, make_optimizer,  # noqa: E402
                                 train_step)

method = sys.argv[1] if len(sys.argv) > 1 else "atf"
net = sys.argv[2] if len(sys.argv) > 2 else "res101"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = torch.device("cuda", 0)
if method == "atf":
    from tlod.data.imdb import VOC_CLASSES
    model = build_model(method, dev, net, classes=VOC_CLASSES, dataset="pascal_voc")
else:
    model = build_model(method, dev, net)
opt = make_optimizer(model, 2e-3, clip=10.0)
data = SyntheticCityscapes(dev, H=600, W=1200, seed=1)
for _ in range(2):
    train_step(model, opt, data.next())
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
             with_stack=True) as prof:
    for _ in range(steps):
        train_step(model, opt, data.next())
    torch.cuda.synchronize()
rows = []
for e in prof.key_averages(group_by_stack_n=6):
    dt = getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)
    if dt <= 0 or e.key.startswith("tlod") or "ProfilerStep" in e.key:
        continue
    frames = [f for f in (e.stack or []) if "tlod/" in f or "tlod\\" in f]
    rows.append((dt / steps, e.count / steps, e.key, frames[:2]))
rows.sort(key=lambda r: -r[0])
tot = sum(r[0] for r in rows)
print(f"torch-side device time per step: {tot / 1e3:.2f} ms")
for dt, n, k, fr in rows[:30]:
    print(f"{dt / 1e3:7.3f} ms {n:6.1f}x  {k[:50]:50s}  {' <- '.join(f.split('/tlod/')[-1] for f in fr)}")
# the glue ops by input shape (their call sites: grep the shapes)
print("-- by input shape: copy_ / mm / add_ / cat / elementwise")
srows = []
for e in prof.key_averages(group_by_input_shape=True):
    dt = getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)
    if dt <= 0 or e.key not in ("aten::copy_", "aten::mm", "aten::add_", "aten::cat", "aten::addmm",
                                "aten::mul", "aten::fill_", "aten::zero_", "aten::sum"):
        continue
    srows.append((dt / steps, e.count / steps, e.key, str(e.input_shapes)[:110]))
srows.sort(key=lambda r: -r[0])
for dt, n, k, sh in srows[:40]:
    print(f"{dt / 1e3:7.3f} ms {n:6.1f}x  {k:14s} {sh}")
