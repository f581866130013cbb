"""One conv layer of the real network, identical f32 inputs: device vs fp64 bias."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle.daf_step import synthetic_batch  # noqa: E402
from tlod import conv as tc  # noqa: E402
from tlod.detector.train import build_daf_vgg16  # noqa: E402

m = build_daf_vgg16("cuda", seed=0)
x = synthetic_batch(192, 320, seed=1)[0].double()
w0, b0 = m.RCNN_base[0].weight.detach(), m.RCNN_base[0].bias.detach()
x1 = F.relu(F.conv2d(x, w0.double().cpu(), b0.double().cpu(), padding=1))  # layer-1 output (exact)
w = m.RCNN_base[2].weight.detach()


def st(a, b):
    e = a.double().cpu() - b
    return f"rel {float(e.norm() / b.norm()):.2e} bias {float((e * b).sum() / (b * b).sum()):+.2e}"


for name, inp in (("real", x1.float()), ("real*0.37", (x1 * 0.37).float()),
                  ("relu(randn)", torch.relu(torch.randn(x1.shape)).float())):
    ref = F.conv2d(inp.double(), w.double().cpu(), padding=1)
    for math in ("bf16x6", "f32"):
        y = tc.conv_fwd(inp.cuda(), w, None, False, math=math)
        print(name, math, st(y, ref))
    print(name, "miopen", st(F.conv2d(inp.cuda(), w, padding=1), ref))
    print(name, "cpu", st(F.conv2d(inp, w.cpu(), padding=1), ref))
