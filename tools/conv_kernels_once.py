"""Run conv3_3-shaped fwd / dgrad / wgrad a few times (for rocprofv3 --pmc passes).
usage: conv_kernels_once.py [math] [N C H W]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch
from tlod import conv as tc
m = sys.argv[1] if len(sys.argv) > 1 else "f32"
N, C, H, W = (int(v) for v in sys.argv[2:6]) if len(sys.argv) > 5 else (2, 256, 150, 250)
x = torch.randn(N, C, H, W, device="cuda"); g = torch.randn(N, C, H, W, device="cuda")
w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
wk = tc.pack_fwd(w) if m == "f32" else tc.pack_bs(w, False)
wd = tc.pack_dgrad(w) if m == "f32" else tc.pack_bs(w, True)
for _ in range(3):
    tc.conv_fwd(x, w, None, True, wk=wk, math=m); tc.conv_dgrad(g, w, wd=wd, math=m)
    tc.conv_wgrad(g, x, 3, math=m)
torch.cuda.synchronize()
