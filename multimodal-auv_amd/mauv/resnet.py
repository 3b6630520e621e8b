"""ResNet-50 v1.5 trunk with torchvision's module names (state_dict-compatible).

The reference builds its trunks with ``torchvision.models.resnet50`` (models/base_models.py:15,
models/model_utils.py:57) — torchvision is not part of this framework's runtime, so the trunk
is declared here: Bottleneck v1.5 (stride on the 3x3), [3, 4, 6, 3], expansion 4,
BatchNorm eps 1e-5 / momentum 0.1, torchvision's init.  Only the *structure and parameters*
live in these modules; execution is the MC-batched engine (mauv.engine), which compiles
the trunk into a fixed schedule of HIP launches.
"""
import torch
import torch.nn as nn

from .layers import is_bayesian


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


class ResNet(nn.Module):
    """torchvision-compatible ResNet-50 whose forward runs on the HIP engine."""

    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, in_channels=3):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(in_channels, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                yield blk

    def has_classifier(self):
        return is_bayesian(self.fc)

    def forward(self, x):
        """x [B,C,H,W] -> features [B,2048] (fc = Identity) or logits [B,C] (Bayesian fc).
        One MC sample, differentiable, BN in the module's train/eval mode."""
        from .engine import run_trunk_mc
        return run_trunk_mc(self, x, 1)[0]

    def mc_forward(self, x, num_mc):
        """All ``num_mc`` MC samples in one batched launch per layer: [num_mc, B, out]."""
        from .engine import run_trunk_mc
        return run_trunk_mc(self, x, num_mc)


def resnet50(weights=None, **kwargs):
    """torchvision signature; ``weights`` cannot be fetched offline (synthetic init)."""
    return ResNet((3, 4, 6, 3), **kwargs)
