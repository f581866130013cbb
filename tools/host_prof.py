"""cProfile of the host side of training steps (where the Python enqueue time goes).
usage: python tools/host_prof.py [steps] [net] [method] [top]"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.detector.train import (SyntheticCityscapes, build_model, make_optimizer,  # noqa: E402
                                 train_step)

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
net = sys.argv[2] if len(sys.argv) > 2 else "vgg16"
method = sys.argv[3] if len(sys.argv) > 3 else "daf"
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
dev = torch.device("cuda", 0)
model = build_model(method, dev, net)
opt = make_optimizer(model, 2e-3)
data = SyntheticCityscapes(dev, H=600, W=1200, seed=1)
for _ in range(3):
    train_step(model, opt, data.next())
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    train_step(model, opt, data.next())
pr.disable()
torch.cuda.synchronize()
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(top)
    print(f"==== {net} {method}, {steps} steps, sorted by {key}")
    print(s.getvalue())
