"""Locate wrong entries of the split-bf16 wgrad vs fp64 on a few shapes (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.conv import conv_wgrad  # noqa: E402

for (N, Cin, Cout, H, W) in [(2, 64, 128, 37, 75), (1, 64, 128, 37, 75), (1, 16, 32, 8, 16),
                             (1, 16, 32, 9, 33), (2, 256, 256, 30, 40)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, Cin, H, W, generator=g)
    gy = torch.randn(N, Cout, H, W, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, 3, 3), gy.double(), padding=1)
    dw = conv_wgrad(gy.cuda(), x.cuda(), 3, math="bf16x6").double().cpu()
    err = (dw - ref).abs()
    bad = err > 1e-4 * ref.abs().max()
    nrm = float((dw - ref).norm() / ref.norm())
    print(f"N={N} Cin={Cin} Cout={Cout} {H}x{W}: normwise {nrm:.2e}, bad {int(bad.sum())}/{bad.numel()}")
    if bad.any():
        idx = bad.nonzero()
        co = idx[:, 0].unique()
        ci = idx[:, 1].unique()
        print("  co:", co[:20].tolist(), "n=", len(co))
        print("  ci:", ci[:20].tolist(), "n=", len(ci))
        taps = (idx[:, 2] * 3 + idx[:, 3]).unique()
        print("  taps:", taps.tolist())
        for t in idx[:5].tolist():
            print("  ", t, float(dw[tuple(t)]), float(ref[tuple(t)]))
