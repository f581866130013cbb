"""Oracle: ResNet101 backbone/head in plain torch-CPU fp32 (test infrastructure only).

A restatement of lib/DAF/resnet.py:64-288 (caffe-style Bottleneck with the stride on the
1x1 conv1, maxpool ceil_mode, RCNN_base = conv1..layer3, RCNN_top = layer4, frozen BN in
eval mode) with the same module names, so a device model's state_dict loads into it.
"""
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    # activation sites (oracle.daf_step.forced_relu), set by name_sites(): the gradient
    # bars evaluate fp64 references in a recorded activation pattern
    forced, site = None, None

    def _relu(self, tag, x):
        if self.forced is None:
            return self.relu(x)
        from .daf_step import forced_relu
        return forced_relu(self.forced, f"{self.site}.{tag}", x)

    def forward(self, x):  # resnet.py:80-102
        residual = x
        out = self._relu("r1", self.bn1(self.conv1(x)))
        out = self._relu("r2", self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            residual = self.downsample(x)
        out = out + residual
        return self._relu("r3", out)


def _make_layer(inplanes, planes, blocks, stride=1):
    downsample = None
    if stride != 1 or inplanes != planes * 4:
        downsample = nn.Sequential(
            nn.Conv2d(inplanes, planes * 4, kernel_size=1, stride=stride, bias=False),
            nn.BatchNorm2d(planes * 4))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * 4, planes))
    return nn.Sequential(*layers)


def resnet101_parts(fixed_blocks=1):
    base = nn.Sequential(nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False),
                         nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                         nn.MaxPool2d(kernel_size=3, stride=2, padding=0, ceil_mode=True),
                         _make_layer(64, 64, 3), _make_layer(256, 128, 4, stride=2),
                         _make_layer(512, 256, 23, stride=2))
    top = nn.Sequential(_make_layer(1024, 512, 3, stride=2))
    for p in list(base[0].parameters()) + list(base[1].parameters()):
        p.requires_grad = False
    for idx in range(4, 4 + fixed_blocks):
        for p in base[idx].parameters():
            p.requires_grad = False
    for m in list(base.modules()) + list(top.modules()):
        if isinstance(m, nn.BatchNorm2d):
            for p in m.parameters():
                p.requires_grad = False
    return base, top


def bn_eval(module):
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.eval()


def name_sites(seq, forced, prefix):
    """Give every Bottleneck under ``seq`` the activation sites ``{prefix}.{i}.{j}.r1/r2/r3``
    (i: index in ``seq``, j: block index) backed by the ``forced`` dict."""
    for i, layer in enumerate(seq):
        if isinstance(layer, nn.Sequential):
            for j, blk in enumerate(layer):
                if isinstance(blk, Bottleneck):
                    blk.forced, blk.site = forced, f"{prefix}.{i}.{j}"
