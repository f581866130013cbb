"""VGG16 backbone and head for the DAF/MAF/ATF detectors (lib/DAF/vgg16.py:20-71).

``RCNN_base`` keeps torchvision vgg16().features[:-1] indices (so state_dict keys are
``RCNN_base.{0,2,5,...}.weight/bias`` as in the reference) with every conv+ReLU pair
fused into one libtlod conv (the ReLU slots become nn.Identity).  Layers 0-9 (conv1_x,
conv2_x) are frozen (vgg16.py:52-53).  ``RCNN_top`` = classifier[:-1]:
Linear(25088,4096) ReLU Dropout Linear(4096,4096) ReLU Dropout (tlod.linear: split-bf16
GEMMs in libtlod).
"""
import torch.nn as nn

from ..conv import Conv2d, vgg_init_
from ..linear import FcTop, Linear

# split points (shared frozen prefix end, conv3 end, conv4 end) of RCNN_base for the MAF /
# ATF taps: conv3 = features[:16], conv34 = [16:23], conv45 = [23:-1] (lib/MAF/vgg16.py:84-86)
VGG16_SPLITS = (10, 16, 23)

# torchvision vgg16 cfg "D"
VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512]


def vgg16_base(frozen_layers=10, fuse_pools=(1, 2)):
    """RCNN_base with the max-pools listed in ``fuse_pools`` (1-4, in order) folded into the
    preceding conv module (Conv2d.pool; the MaxPool2d slot becomes nn.Identity, so indices and
    state_dict keys are unchanged).  Pools 1/2 follow frozen convs whose output feeds nothing
    else (the conv epilogue pools, the full map is never written); pools 3/4 fold only where
    no DA tap reads the conv3 / conv4 outputs (DAF), routing the backward through the fused
    argmax + ReLU kernel."""
    layers, cin, npool = [], 3, 0
    for v in VGG16_CFG:
        if v == "M":
            npool += 1
            if npool in fuse_pools:
                layers[-2].pool = True
                layers.append(nn.Identity())
            else:
                layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            conv = Conv2d(cin, v, 3, relu=True)
            vgg_init_(conv)
            layers += [conv, nn.Identity()]  # index of the fused ReLU stays occupied
            cin = v
    base = nn.Sequential(*layers)  # features[:-1]: the last max-pool is not used
    for i in range(frozen_layers):
        for p in base[i].parameters():
            p.requires_grad = False
    return base


def vgg16_top():
    fc6, fc7 = Linear(512 * 7 * 7, 4096), Linear(4096, 4096)
    for m in (fc6, fc7):  # torchvision VGG Linear init
        m.weight.data.normal_(0, 0.01)
        m.bias.data.zero_()
    return FcTop(fc6, nn.ReLU(True), nn.Dropout(), fc7, nn.ReLU(True), nn.Dropout())
