import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch, torch.nn.functional as F
from tlod.conv import ConvFunction, conv_dgrad, conv_wgrad, relu_bwd_bias
def rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm())
for (N, Cin, Cout, H, W) in [(1,512,512,37,62), (1,256,256,30,40), (1,512,512,32,64), (2,512,512,37,62)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5
    gy = torch.randn(N, Cout, H, W, generator=g)
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1); yr.backward(gy.double())
    dx = conv_dgrad(gy.cuda(), w.cuda())
    dw = conv_wgrad(gy.cuda(), x.cuda(), 3)
    gg, db = relu_bwd_bias(gy.cuda(), None, True)
    print((N,Cin,Cout,H,W), "dx", rel(dx, xr.grad), "dw", rel(dw, wr.grad), "db", rel(db, gy.double().sum((0,2,3))))
    e = (dw.cpu().double() - wr.grad).abs().sum((1,2,3))
    print("  dw bad co:", (e > 1e-3 * e.max()).nonzero().view(-1)[:20].tolist() if rel(dw, wr.grad) > 1e-4 else "-")
