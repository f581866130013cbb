"""Run conv3_3-shaped fwd / dgrad / wgrad a few times (for rocprofv3 --pmc passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch
from tlod import conv as tc
N, C, H, W = 2, 256, 150, 250
x = torch.randn(N, C, H, W, device="cuda"); g = torch.randn(N, C, H, W, device="cuda")
w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
wk, wd = tc.pack_fwd(w), tc.pack_dgrad(w)
for _ in range(3):
    tc.conv_fwd(x, w, None, True, wk=wk); tc.conv_dgrad(g, w, wd=wd); tc.conv_wgrad(g, x, 3)
torch.cuda.synchronize()
