"""PMC calibration run for the conv kernels' access widths (MI355X_MICROARCH.md: only
16-B/lane streaming reads are calibrated): conv1_2-shaped split-bf16 forward, 2x64x600x1200
in (368.6 MB) -> 368.6 MB out, input and output far beyond the 256 MiB Infinity Cache."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod import conv as tc  # noqa: E402

x = torch.randn(2, 64, 600, 1200, device="cuda")
w = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
wp = tc.pack_bs(w, False)
g = torch.randn(2, 64, 600, 1200, device="cuda")
for _ in range(3):
    tc.conv_fwd(x, w, None, True, wk=wp, math="bf16x6")
    tc.conv_wgrad(g, x, 3, math="bf16x6")
torch.cuda.synchronize()
