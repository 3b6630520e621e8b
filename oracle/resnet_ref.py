"""Oracle: torchvision ResNet-50 v1.5 restated on torch-CPU (TEST INFRASTRUCTURE ONLY).

torchvision is not installed in the image and is not vendored by the reference; the
reference uses it at ``models/base_models.py:2,15`` (``resnet50(weights=IMAGENET1K_V1)``)
and ``models/model_utils.py:3,57-61``.  Restated from torchvision's published
architecture: Bottleneck v1.5 (stride on the 3x3), layers [3, 4, 6, 3], expansion 4,
BatchNorm eps 1e-5 momentum 0.1, stem 7x7/2 pad 3 + maxpool 3x3/2 pad 1, adaptive avg
pool, ``fc`` Linear(2048, 1000).  Module names match torchvision exactly so the
state_dict keys (``layer1.0.conv1.weight``, ``layer1.0.downsample.0.weight`` ...) are the
reference's.

Weights: ImageNet weights cannot be fetched (no network) — ``weights`` is accepted and
ignored; parameters are initialised the torchvision way (kaiming_normal fan_out for
convs, BN gamma=1/beta=0, default Linear init) from the ambient torch RNG, so callers
seed with ``torch.manual_seed`` for determinism (synthetic weights; documented in
DESIGN.md).
"""
import math

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, kernel_size=1, stride=1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = out + identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, kernel_size=1,
                          stride=stride, bias=False),
                nn.BatchNorm2d(planes * Bottleneck.expansion),
            )
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


class ResNet50_Weights:
    """Stand-in for ``torchvision.models.ResNet50_Weights`` (enum value only)."""
    IMAGENET1K_V1 = "IMAGENET1K_V1"


def resnet50(weights=None, **kwargs):
    """torchvision ``resnet50`` restated; ``weights`` ignored (offline: synthetic init)."""
    return ResNet((3, 4, 6, 3), **kwargs)


def conv_macs(model: nn.Module, x_shape):
    """Multiply-accumulates of every Conv2d/Linear for one input of ``x_shape`` (C,H,W)."""
    macs = 0
    hooks = []

    def conv_hook(m, inp, out):
        nonlocal macs
        k = m.in_channels // m.groups * m.kernel_size[0] * m.kernel_size[1]
        macs += out.numel() // out.shape[0] * k

    def lin_hook(m, inp, out):
        nonlocal macs
        macs += m.in_features * m.out_features

    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, nn.Linear):
            hooks.append(m.register_forward_hook(lin_hook))
    with torch.no_grad():
        model.eval()(torch.zeros(1, *x_shape))
    for h in hooks:
        h.remove()
    return macs
