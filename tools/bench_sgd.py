"""Microbenchmark: the fused clip + SGD step (tlod_sgd_clip_f32) over DAF-VGG16's trainable
parameter shapes (~137 M floats), HIP events around optimizer.step()."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.detector.train import build_model, make_optimizer  # noqa: E402

dev = torch.device("cuda", 0)
model = build_model("daf", dev, "vgg16")
opt = make_optimizer(model, 2e-3, clip=10.0)
n = 0
for p in opt.params:
    g = opt.arena.view(p) if opt.arena is not None else torch.empty_like(p)
    g.normal_()
    p.grad = g
    n += p.numel()
for _ in range(3):
    opt.step()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
it = 20
for _ in range(it):
    opt.step()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / it
print(f"params {n / 1e6:.1f} M, step {ms:.3f} ms, {24 * n / (ms * 1e-3) / 1e12:.2f} TB/s "
      f"(6 x 4 B per parameter: g read twice, p and buf read + written)")
