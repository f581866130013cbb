"""Which parameters' gradients reach the gradient arena by a copy (not written into their
slot by the backward): one DAF step, names printed with their sizes.
usage: python tools/arena_copies.py [net] [method]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.detector.train import SyntheticCityscapes, build_model, make_optimizer, train_step  # noqa: E402
from tlod import grads  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "res101"
method = sys.argv[2] if len(sys.argv) > 2 else "daf"
dev = torch.device("cuda", 0)
model = build_model(method, dev, net)
opt = make_optimizer(model, 2e-3, clip=10.0)
data = SyntheticCityscapes(dev, H=600, W=1200, seed=1)
train_step(model, opt, data.next())
names = {p: n for n, p in model.named_parameters()}
copied = []
orig = grads.GradArena._on_grad


def spy(self, p):
    g = p.grad
    off = self.offset[p]
    if g.data_ptr() != self.flat.data_ptr() + 4 * off:
        copied.append((names.get(p, "?"), tuple(p.shape)))
    return orig(self, p)


grads.GradArena._on_grad = spy
for h in opt.arena.hooks:
    h.remove()
opt.arena.hooks = [p.register_post_accumulate_grad_hook(opt.arena._on_grad) for p in opt.arena.params]
train_step(model, opt, data.next())
torch.cuda.synchronize()
print(len(copied), "copied gradients")
for n, s in copied:
    print(n, s)
