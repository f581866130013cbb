import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "transfer-learning-library-for-object-detection_amd"))
import torch, torch.nn.functional as F
from tlod import conv as tc
torch.manual_seed(0)
for (N, Cin, Cout, H, W) in [(1,512,512,37,62),(1,512,128,37,62),(1,128,512,37,62),(1,512,512,32,64),(1,512,512,37,64),(1,512,512,36,62),(1,256,512,37,62),(1,384,512,37,62),(1,512,256,37,62)]:
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) * (2.0 / (Cin * 9)) ** 0.5
    y = tc.conv_fwd(x.cuda(), w.cuda(), None, False).cpu().double()
    r = F.conv2d(x.double(), w.double(), padding=1)
    e = (y - r).abs()
    bad = (e > 1e-3 * r.abs().max())
    idx = bad.nonzero()
    print((N, Cin, Cout, H, W), "nrm", float((y-r).norm()/r.norm()), "bad", int(bad.sum()),
          "co", sorted(set(idx[:,1].tolist()))[:10], "h", sorted(set(idx[:,2].tolist()))[:20], "w", sorted(set(idx[:,3].tolist()))[:40])
