"""Run the conv3_3-shaped fwd (f32 or split-bf16 math) a few times (for rocprofv3 --pmc)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch
from tlod import conv as tc
m = sys.argv[1] if len(sys.argv) > 1 else "bf16x6"
N, C, H, W = 2, 256, 150, 250
x = torch.randn(N, C, H, W, device="cuda")
w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
wk = tc.pack_bs(w, False) if m != "f32" else tc.pack_fwd(w)
for _ in range(3):
    tc.conv_fwd(x, w, None, True, wk=wk, math=m)
torch.cuda.synchronize()
