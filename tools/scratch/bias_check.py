"""Coherent (scale) bias of conv / GEMM results vs fp64: <err, ref> / <ref, ref>."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from tlod import conv as tc  # noqa: E402
from tlod.linear import gemm  # noqa: E402

torch.manual_seed(0)


def stats(a, b):
    e = a.double().cpu() - b
    return f"rel {float(e.norm() / b.norm()):.2e} bias {float((e * b).sum() / (b * b).sum()):+.2e}"


N, C, H, W, K = 2, 256, 48, 80, 256
x = torch.relu(torch.randn(N, C, H, W))
w = torch.randn(K, C, 3, 3) * (2.0 / (9 * C)) ** 0.5
ref = F.conv2d(x.double(), w.double(), padding=1)
xd, wd = x.cuda(), w.cuda()
print("fwd cpu   ", stats(F.conv2d(x, w, padding=1), ref))
print("fwd miopen", stats(F.conv2d(xd, wd, padding=1), ref))
for m in ("bf16x6", "f32", "bf16x3"):
    print("fwd", m, stats(tc.conv_fwd(xd, wd, None, False, math=m), ref))
gy = torch.randn(N, K, H, W) * 1e-4
refd = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1)
for m in ("bf16x6", "f32"):
    print("dgrad", m, stats(tc.conv_dgrad(gy.cuda(), wd, math=m), refd))
print("dgrad miopen", stats(torch.nn.grad.conv2d_input(x.shape, wd, gy.cuda(), padding=1), refd))
refw = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=1)
for m in ("bf16x6", "f32"):
    print("wgrad", m, stats(tc.conv_wgrad(gy.cuda(), xd, 3, math=m), refw))
print("wgrad miopen", stats(torch.nn.grad.conv2d_weight(xd, w.shape, gy.cuda(), padding=1), refw))
M, Nn, Kk = 556, 4096, 25088
a = torch.relu(torch.randn(M, Kk))
b = torch.randn(Nn, Kk) * 0.01
r = a.double() @ b.double().t()
print("gemm bf16x6", stats(gemm(a.cuda(), b.cuda(), M, Nn, Kk, 1, 1), r))
print("gemm hipblas", stats(a.cuda() @ b.cuda().t(), r))
print("gemm cpu", stats(a @ b.t(), r))
