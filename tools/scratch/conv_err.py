"""Per-layer arithmetic error vs fp64: split-bf16 / f32-MFMA convs and GEMMs vs CPU fp32."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from tlod import conv as tc  # noqa: E402
from tlod.linear import gemm  # noqa: E402

torch.manual_seed(0)


def rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm())


for (N, C, H, W, K) in [(2, 256, 48, 80, 256), (2, 512, 24, 40, 512), (2, 64, 96, 160, 128)]:
    x = torch.relu(torch.randn(N, C, H, W))
    w = torch.randn(K, C, 3, 3) * (2.0 / (9 * C)) ** 0.5
    ref = F.conv2d(x.double(), w.double(), padding=1)
    cpu = F.conv2d(x, w, padding=1)
    xd, wd = x.cuda(), w.cuda()
    r = {"cpu_f32": rel(cpu, ref)}
    for m in ("bf16x6", "f32"):
        r[m] = rel(tc.conv_fwd(xd, wd, None, False, math=m), ref)
    r["miopen_f32"] = rel(F.conv2d(xd, wd, padding=1), ref)
    gy = torch.randn(N, K, H, W)
    refw = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=1)
    r["wgrad_cpu"] = rel(torch.nn.grad.conv2d_weight(x, w.shape, gy, padding=1), refw)
    for m in ("bf16x6", "f32"):
        r["wgrad_" + m] = rel(tc.conv_wgrad(gy.cuda(), xd, 3, math=m), refw)
    print((N, C, H, W, K), {k: f"{v:.2e}" for k, v in r.items()})

for (M, N, K) in [(556, 4096, 25088), (556, 1024, 4096)]:
    a = torch.relu(torch.randn(M, K))
    b = torch.randn(N, K) * 0.01
    ref = a.double() @ b.double().t()
    r = {"cpu_f32": rel(a @ b.t(), ref), "bf16x6": rel(gemm(a.cuda(), b.cuda(), M, N, K, 1, 1), ref),
         "hipblas_f32": rel(a.cuda() @ b.cuda().t(), ref)}
    print((M, N, K), {k: f"{v:.2e}" for k, v in r.items()})
