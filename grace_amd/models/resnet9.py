"""cifar10-fast / DAWNBench ResNet-9 (reference examples/dist/CIFAR10-dawndist/dawn.py:26-63).

prep conv(64) -> layer1 conv(128)+pool+residual -> layer2 conv(256)+pool -> layer3
conv(512)+pool+residual -> global max-pool -> linear(10, no bias) scaled by 0.125.  The only
published performance number in the reference tree is this network's 24-epoch CIFAR-10 run
(79 s incl. validation, ~74 s DAWNBench train time on one V100:
examples/dist/CIFAR10-dawndist/README.md:17, 24-26).
"""
import torch.nn as nn

from ..ops.bnact import BatchNormAct2d
from ..ops.pool import MaxPool2dNHWC


def conv_bn(cin, cout):
    # conv -> BN -> ReLU; BN+ReLU is one fused op (grace_amd/ops/bnact.py)
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), BatchNormAct2d(cout, relu=True))


class Residual(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.res = nn.Sequential(conv_bn(c, c), conv_bn(c, c))

    def forward(self, x):
        return x + self.res(x)


class ResNet9(nn.Module):
    def __init__(self, classes=10, weight=0.125):
        super().__init__()
        self.net = nn.Sequential(
            conv_bn(3, 64),
            conv_bn(64, 128), MaxPool2dNHWC(2), Residual(128),
            conv_bn(128, 256), MaxPool2dNHWC(2),
            conv_bn(256, 512), MaxPool2dNHWC(2), Residual(512),
            nn.AdaptiveMaxPool2d(1), nn.Flatten(), nn.Linear(512, classes, bias=False))
        self.weight = weight

    def forward(self, x):
        return self.net(x) * self.weight


def resnet9(classes=10):
    return ResNet9(classes)
