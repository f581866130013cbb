import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch, torch.nn.functional as F
from tlod.conv import ConvFunction
dev = "cuda"
N, Cin, Cout, H, W, KS = 1, 512, 512, 37, 62, 3
g = torch.Generator().manual_seed(N * 1000 + Cin + Cout + H)
x = torch.randn(N, Cin, H, W, generator=g)
w = torch.randn(Cout, Cin, KS, KS, generator=g) * (2.0 / (Cin * KS * KS)) ** 0.5
b = torch.randn(Cout, generator=g)
def rel(a, b_):
    a = a.detach().double().cpu(); b_ = b_.detach().double().cpu()
    return float((a - b_).norm() / b_.norm()), float((a-b_).abs().max()), float(b_.abs().max())
for relu in (False, True):
    xd, wd, bd = (t.to(dev).requires_grad_(True) for t in (x, w, b))
    y = ConvFunction.apply(xd, wd, bd, relu)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, padding=KS // 2)
    if relu: yr = F.relu(yr)
    print(relu, "y", rel(y, yr))
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev)); yr.backward(gy.double())
    print(relu, "dx", rel(xd.grad, xr.grad), "dw", rel(wd.grad, wr.grad), "db", rel(bd.grad, br.grad))
    if relu:
        m1 = (y.detach().cpu() > 0); m2 = (yr.detach() > 0)
        print("mask mismatches", int((m1 != m2).sum()), "zeros gpu", int((y==0).sum()))
