"""Where the source-only step's gradient error enters: forward activations and their
gradients (device vs fp64 in the device's activation pattern; torch-GPU fp32 alongside)."""
import copy
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import arm_device_taps, device_forced, record_pattern, run_in_pattern  # noqa: E402
from oracle.frcnn_step import OracleFRCNN, total_loss  # noqa: E402
from tlod.config import cfg, setup_training_cfg  # noqa: E402
from tlod.data.imdb import VOC_CLASSES  # noqa: E402
from tlod.data.loader import collate, roibatchLoader  # noqa: E402
from tlod.data.roidb import combined_roidb  # noqa: E402
from tlod.data.synthetic import synthetic_voc  # noqa: E402
from tlod.detector.train import build_model  # noqa: E402

root = tempfile.mkdtemp()
synthetic_voc(root, [(600, 1000)], VOC_CLASSES, seed=3, n_objects=6)
setup_training_cfg("vgg16", "pascal_voc")
imdb, roidb, rl, ri = combined_roidb("voc_2007_trainval", root)
ld = roibatchLoader(roidb, rl, ri, 1, imdb.num_classes, training=True)
m = build_model("faster_rcnn", "cuda", "vgg16", classes=VOC_CLASSES, dataset="pascal_voc")
for mod in m.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.p = 0.0
np.random.seed(3)
data, im_info, gt, num = collate([ld[0]])


def grab(mod, store, name):
    def fwd(_m, _i, out):
        out.retain_grad()
        store[name] = out
    return mod.register_forward_hook(fwd)


dv = {}
grab(m.RCNN_base, dv, "base")
grab(m.RCNN_top, dv, "fc7")
grab(m.RCNN_top[0], dv, "fc6pre")
grab(m.RCNN_roi_align, dv, "pooled")
m.replay_rng = np.random.RandomState(3)
m.capture = {}
taps = arm_device_taps(m)
out = m(data, im_info, gt, num)
m.total_loss(out).backward()
s_rois = m.capture["s_rois"].cpu().numpy()
o = OracleFRCNN(21, scales=(8, 16, 32), dropout=0.0).train()
o.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=True)
cpu = (data.cpu(), im_info.cpu(), gt.cpu())


def run(model, batch, store):
    hs = [grab(model.RCNN_base[29], store, "base"), grab(model.RCNN_top, store, "fc7"),
          grab(model.RCNN_top[0], store, "fc6pre")]
    loss = total_loss(model(*batch, np.random.RandomState(3), rois_override=s_rois))
    loss.backward()
    for h in hs:
        h.remove()


o64 = copy.deepcopy(o).double()
s64 = {}
run_in_pattern(o64, device_forced(taps), lambda: run(o64, tuple(t.double() for t in cpu), s64))
og = copy.deepcopy(o).cuda()
sg = {}
own = record_pattern(og, lambda: run(og, tuple(t.cuda() for t in cpu), sg))
o64g = copy.deepcopy(o).double()
s64g = {}
run_in_pattern(o64g, own, lambda: run(o64g, tuple(t.double() for t in cpu), s64g))


def st(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    e = a - b
    return f"rel {float(e.norm() / b.norm()):.2e} bias {float((e * b).sum() / (b * b).sum()):+.2e}"


for name in ("base", "fc6pre", "fc7"):
    print(f"{name:7s} fwd  dev {st(dv[name], s64[name])} | gpu32 {st(sg[name], s64g[name])}")
    print(f"{name:7s} grad dev {st(dv[name].grad, s64[name].grad)} | gpu32 {st(sg[name].grad, s64g[name].grad)}")
gp = dict(m.named_parameters())
for k in ("RCNN_cls_score.weight", "RCNN_top.3.weight", "RCNN_top.0.weight", "RCNN_base.28.weight",
          "RCNN_base.10.weight"):
    print(k, "dev", st(gp[k].grad, dict(o64.named_parameters())[k].grad), "| gpu32",
          st(dict(og.named_parameters())[k].grad, dict(o64g.named_parameters())[k].grad))
