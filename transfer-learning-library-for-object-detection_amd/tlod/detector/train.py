"""The DAF training step (methods/DAF/DAF_train.py:353-408) on the tlod path, plus the
synthetic Cityscapes->Foggy batch source used by bench.py / smoke().

Per step (one source + one target image): forward -> loss sum with lamda * DA terms
(:397-400) -> backward -> clip_gradient(10) for VGG16 (:406-407, here device-side with
no .item()) -> SGD(momentum 0.9; biases 2x lr, no weight decay; weights lr, wd 5e-4)
(:311-325).  Optional gradient all-reduce hook (tlod.dist) runs inside backward.
"""
import math

import numpy as np
import torch

from ..config import cfg, setup_training_cfg

from ..data.imdb import CITYSCAPE_CLASSES as CITYSCAPES_CLASSES  # cityscape.py:51-54


METHODS = ("faster_rcnn", "daf", "maf", "atf")


def build_model(method, device, net="vgg16", classes=CITYSCAPES_CLASSES, seed=0,
                dataset="cityscape"):
    """<method>.<net>(classes).create_architecture() (methods/<M>/<M>_train.py), random
    init (the pretrained caffe weights are external downloads).  method "faster_rcnn" is
    the source-only detector (lib/model/faster_rcnn, methods/faster_rcnn)."""
    if method not in METHODS:
        raise ValueError(f"unknown method {method!r} (have {METHODS})")
    if net not in ("vgg16", "res101"):
        raise ValueError(f"unknown backbone {net!r}")
    import importlib
    mod = importlib.import_module(".faster_rcnn" if method == "faster_rcnn" else f"..da.{method}",
                                  __package__)
    if net == "res101" and not hasattr(mod, "resnet"):
        raise NotImplementedError(f"{method} with ResNet101")
    setup_training_cfg(net, dataset)
    torch.manual_seed(seed)
    if net == "vgg16":
        m = mod.vgg16(classes, pretrained=False, class_agnostic=False)
    else:
        m = mod.resnet(classes, 101, pretrained=False, class_agnostic=False)
    m.create_architecture()
    m.net = net
    return m.to(device).train()


def build_daf_vgg16(device, classes=CITYSCAPES_CLASSES, seed=0):
    return build_model("daf", device, "vgg16", classes, seed)


def make_optimizer(model, lr, momentum=None, weight_decay=None, double_bias=None, bias_decay=None,
                   fused=True, clip=None):
    """DAF_train.py:311-325 param groups (collapsed to two groups — same update).
    fused=True: libtlod's fused clip_gradient(clip) + SGD (tlod.optim.FusedSGDClip).
    clip None: 10 for VGG16, none for ResNet101 (DAF_train.py:406-407)."""
    if clip is None:
        clip = default_clip(model)
    momentum = cfg.TRAIN.MOMENTUM if momentum is None else momentum
    wd = cfg.TRAIN.WEIGHT_DECAY if weight_decay is None else weight_decay
    double_bias = cfg.TRAIN.DOUBLE_BIAS if double_bias is None else double_bias
    bias_decay = cfg.TRAIN.BIAS_DECAY if bias_decay is None else bias_decay
    biases, weights = [], []
    for k, v in model.named_parameters():
        if v.requires_grad:
            (biases if "bias" in k else weights).append(v)
    groups = [{"params": weights, "lr": lr, "weight_decay": wd},
              {"params": biases, "lr": lr * (double_bias + 1),
               "weight_decay": wd if bias_decay else 0.0}]
    if fused:
        from ..optim import FusedSGDClip
        return FusedSGDClip(groups, momentum=momentum, clip_norm=clip)
    return torch.optim.SGD(groups, lr=lr, momentum=momentum, foreach=True)


@torch.no_grad()
def clip_gradient_(params, clip_norm):
    """net_utils.py:38-49 without the host sync: total = sqrt(sum ||g||^2);
    g *= clip / max(total, clip)."""
    grads = [p.grad for p in params if p.requires_grad and p.grad is not None]
    if not grads:
        return None
    norms = torch._foreach_norm(grads)
    total = torch.linalg.vector_norm(torch.stack(norms))
    scale = clip_norm / torch.clamp(total, min=clip_norm)
    torch._foreach_mul_(grads, scale)
    return total


class SyntheticCityscapes:
    """Synthetic batches of the reference's input tensors:
    BGR uint8 uniform[0,255] at 600x1200 minus PIXEL_MEANS (NCHW fp32); source gt = 8
    boxes (x1 in [0,W-64), size 32..400, clipped, class 1..8) padded to 50;
    target gt = [1,1,1,1,1] (roibatchLoader.py:217-226).  A small pool of batches is made
    resident on the device up front so the timed loop reads HBM only."""

    def __init__(self, device, H=600, W=1200, G=8, max_gt=50, pool=4, seed=1000, n_classes=8):
        self.device = torch.device(device)
        rng = np.random.default_rng(seed)
        means = torch.tensor(cfg.PIXEL_MEANS.reshape(3), dtype=torch.float32)
        self.batches = []
        for _ in range(pool):
            def img():
                u8 = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8))
                return (u8.float() - means).permute(2, 0, 1).contiguous()[None]
            gt = np.zeros((1, max_gt, 5), np.float32)
            x1 = rng.uniform(0, W - 64, G)
            y1 = rng.uniform(0, H - 64, G)
            w = rng.uniform(32, 400, G)
            h = rng.uniform(32, 400, G)
            gt[0, :G, 0] = x1
            gt[0, :G, 1] = y1
            gt[0, :G, 2] = np.minimum(x1 + w, W - 1)
            gt[0, :G, 3] = np.minimum(y1 + h, H - 1)
            gt[0, :G, 4] = rng.integers(1, n_classes + 1, G)
            info = torch.tensor([[H, W, 600.0 / 1024.0]], dtype=torch.float32)
            d = self.device
            self.batches.append((
                img().to(d), info.to(d), torch.from_numpy(gt).to(d),
                torch.tensor([G], dtype=torch.int64, device=d), torch.ones(1, device=d),
                img().to(d), info.clone().to(d), torch.ones((1, 5), device=d),
                torch.zeros(1, dtype=torch.int64, device=d), torch.zeros(1, device=d)))
        self.i = 0

    def next(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


def daf_loss(out, lamda=0.1):
    from ..da.daf import _fasterRCNN
    return _fasterRCNN.total_loss(out, lamda)


def default_clip(model):
    return 10.0 if getattr(model, "net", "vgg16") == "vgg16" else 0.0


def train_step(model, optimizer, batch, lamda=0.1, clip=None, reducer=None):
    """One DAF/MAF/ATF iteration (the method's own loss sum, model.total_loss); returns the
    loss as a device tensor (no host sync)."""
    from ..optim import FusedSGDClip
    fused = isinstance(optimizer, FusedSGDClip)
    if reducer is not None:
        reducer.zero_grad()  # grads are views into the arena the reducer all-reduces
    else:
        optimizer.zero_grad(set_to_none=True)
    out = model(*batch)
    loss = model.total_loss(out, lamda)
    loss.backward()
    scale = 1.0
    if reducer is not None:
        reducer.finish(scale=not fused)  # SUM all-reduce; the fused step applies 1/world
        scale = reducer.grad_scale
    if fused:
        optimizer.step(grad_scale=scale)  # clip_gradient + SGD fused
    else:
        clip = default_clip(model) if clip is None else clip
        if clip:
            clip_gradient_([p for p in model.parameters()], clip)
        optimizer.step()
    return loss.detach()


def smoke_step(device, method="daf", net="vgg16"):
    """One tiny <method>-<net> forward+backward+update on `device` (used by smoke())."""
    model = build_model(method, device, net)
    opt = make_optimizer(model, 2e-3)
    data = SyntheticCityscapes(device, H=192, W=320, G=4, pool=1, seed=7)
    loss = train_step(model, opt, data.next())
    torch.cuda.synchronize()
    v = float(loss)
    assert math.isfinite(v), f"non-finite {method} loss {v}"
    return v
