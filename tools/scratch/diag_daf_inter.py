"""Diagnostic: intermediate gradients of the DAF step (base features, pooled, fc7) device vs
fp32 / fp64 oracle."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

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


def grab(mod, store, name):
    def fwd(_m, _i, out):
        out.retain_grad()
        store.setdefault(name, []).append(out)
    return mod.register_forward_hook(fwd)


dv = {}
grab(m.RCNN_base, dv, "base")
grab(m.RCNN_top, dv, "fc7")
grab(m.RCNN_roi_align, dv, "pooled")
grab(m.RCNN_instanceDA.dc_ip1, dv, "ip1")
m.replay_rng = np.random.RandomState(3)
m.capture = {}
out = m(*tuple(x.cuda() for x in cpu_batch))
daf_loss(out).backward()
ov = (m.capture["s_rois"].cpu().numpy(), m.capture["t_rois"].cpu().numpy())


def run(model, batch):
    st = {}
    hs = [grab(model.RCNN_base[29], st, "base"), grab(model.RCNN_top, st, "fc7"),
          grab(model.RCNN_instanceDA.dc_ip1, st, "ip1")]
    total_loss(model(batch, np.random.RandomState(3), rois_override=ov)).backward()
    for h in hs:
        h.remove()
    return st


s32 = run(o, cpu_batch)
o64 = copy.deepcopy(o).double()
s64 = run(o64, tuple(t.double() if t.is_floating_point() else t for t in cpu_batch))


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


for name in ("base", "fc7", "ip1"):
    d = dv[name][0]
    n_s = 256
    parts = [d[:1], d[1:]] if name == "base" else [d[:n_s], d[n_s:]]
    for k in range(2):
        dd = parts[k].detach().cpu()
        r32, r64 = s32[name][k], s64[name][k]
        g = d.grad.cpu()
        gp = [g[:1], g[1:]] if name == "base" else [g[:n_s], g[n_s:]]
        print(f"{name}[{k}] fwd dev {rel(dd, r64.detach()):.2e} o32 {rel(r32.detach(), r64.detach()):.2e} | "
              f"grad dev {rel(gp[k], r64.grad):.2e} o32 {rel(r32.grad, r64.grad):.2e}")

# ReLU mask disagreements (pre-activation sign) device vs fp64, fp32 vs fp64
for name in ("ip1",):
    d = dv[name][0].detach().cpu().double()
    r64 = torch.cat([s64[name][0].detach(), s64[name][1].detach()])
    r32 = torch.cat([s32[name][0].detach(), s32[name][1].detach()]).double()
    flips_d = ((d > 0) != (r64 > 0))
    flips_c = ((r32 > 0) != (r64 > 0))
    print(name, "mask flips dev", int(flips_d.sum()), "o32", int(flips_c.sum()),
          "dev flip |z|:", d[flips_d].abs().tolist()[:5], "|z| scale", float(r64.abs().mean()))
