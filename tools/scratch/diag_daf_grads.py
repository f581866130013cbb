"""Diagnostic: DAF step gradient error vs an fp64 oracle run, under the current env knobs."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import grad_errors  # noqa: E402
from oracle.daf_step import OracleDAF, synthetic_batch, total_loss  # noqa: E402
from tlod.detector.train import build_daf_vgg16, daf_loss  # noqa: E402

H, W, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
m = build_daf_vgg16("cuda", seed=seed)
for mod in m.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.p = 0.0
o = OracleDAF(dropout=0.0).train()
o.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=True)
cpu_batch = synthetic_batch(H, W, seed=seed + 1)
if os.environ.get("DIAG_UNBATCHED"):
    t = synthetic_batch(H - 32, W, seed=seed + 5)
    cpu_batch = cpu_batch[:5] + t[5:7] + cpu_batch[7:]
m.replay_rng = np.random.RandomState(3)
m.capture = {}
out = m(*tuple(x.cuda() for x in cpu_batch))
daf_loss(out).backward()
ov = (m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy())
ref = o(cpu_batch, np.random.RandomState(3), rois_override=ov)
total_loss(ref).backward()
o64 = copy.deepcopy(o).double()
for p in o64.parameters():
    p.grad = None
b64 = tuple(t.double() if t.is_floating_point() else t for t in cpu_batch)
total_loss(o64(b64, np.random.RandomState(3), rois_override=ov)).backward()
errs = grad_errors(m.named_parameters(), o, o64)
worst = sorted(errs.items(), key=lambda kv: -kv[1][0] / max(kv[1][1], 2e-6))[:6]
print(os.environ.get("DIAG_TAG", ""), "worst:", [(k, f"{a:.2e}", f"{b:.2e}") for k, (a, b) in worst])
