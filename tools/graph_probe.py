"""Probe: capture one training step in a HIP graph (torch.cuda.CUDAGraph) and time graph
replays against eager steps.  usage: python tools/graph_probe.py [net] [method] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.detector.train import (SyntheticCityscapes, build_model, make_optimizer,  # noqa: E402
                                 train_step)

net = sys.argv[1] if len(sys.argv) > 1 else "vgg16"
method = sys.argv[2] if len(sys.argv) > 2 else "daf"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda", 0)
model = build_model(method, dev, net)
opt = make_optimizer(model, 2e-3, clip=10.0)
data = SyntheticCityscapes(dev, H=600, W=1200, seed=1)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for _ in range(3):
    train_step(model, opt, data.next())
eager = timed(lambda: train_step(model, opt, data.next()))
static = [t.clone() for t in data.next()]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        train_step(model, opt, static)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    loss = train_step(model, opt, static)
torch.cuda.synchronize()


def replay():
    b = data.next()
    for d, x in zip(static, b):
        d.copy_(x)
    g.replay()


graphed = timed(replay)
print(f"{net}/{method}: eager {eager:.2f} ms/step, graph {graphed:.2f} ms/step, loss {float(loss):.4f}")
