"""ResNet family (He et al., 2016) for the synthetic benchmarks.

torchvision is not available in this environment, so the architectures used by the reference
harness (/root/reference/examples/torch/pytorch_synthetic_benchmark.py:86 uses
``torchvision.models.resnet50``) are defined here from the paper: identical layer shapes,
parameter counts (ResNet-50: 25,557,032) and initialisation scheme (Kaiming-normal convs,
BN gamma=1/beta=0).  ``resnet18_cifar`` is the CIFAR-shape variant (3x3 stem, no max-pool)
used by BASELINE config 1.
"""
from __future__ import annotations

from typing import List, Type, Union

import torch
import torch.nn as nn

from ..ops.bnact import BatchNormAct2d, bn_relu_maxpool
from ..ops.bnconv import basic_main, bottleneck_main
from ..ops.conv import Conv1x1F32, conv_bn_act
from ..ops.pool import GlobalAvgPoolFlat, MaxPool2dNHWC
from ..ops.wgrad import Conv2dSplitGrad


def _conv3x3(cin, cout, stride=1):
    # weight gradient on the side stream (ops/wgrad.py), nn.Conv2d state_dict
    return Conv2dSplitGrad(cin, cout, 3, stride=stride, padding=1, bias=False)


def _conv1x1(cin, cout, stride=1):
    # stride-1 1x1 convs are plain GEMMs over channels_last activations: Conv1x1F32 can run them on
    # the hand-written f32 MFMA GEMM (opt-in, GRACE_CONV_MFMA=1; nn.Conv2d state_dict either way)
    if stride == 1:
        return Conv1x1F32(cin, cout)
    return Conv2dSplitGrad(cin, cout, 1, stride=stride, bias=False)


def _down(down: nn.Module, x):
    """The projection shortcut (conv -> BN): the BN statistics may come from the conv's epilogue."""
    if isinstance(down, nn.Sequential) and len(down) == 2 and isinstance(down[1], BatchNormAct2d):
        return conv_bn_act(down[0], down[1], x)
    return down(x)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, down=None):
        super().__init__()
        self.conv1 = _conv3x3(cin, planes, stride)
        self.bn1 = BatchNormAct2d(planes, relu=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = BatchNormAct2d(planes, relu=True)  # relu(bn2(.) + identity), one fused op
        self.downsample = down

    def forward(self, x):
        xm, xs = x if isinstance(x, tuple) else (x, x)
        idt = xs if self.downsample is None else _down(self.downsample, xs)
        out = basic_main(self, xm, idt)  # bn1 applied inside conv2's GEMM (ops/bnconv.py)
        if out is not None:
            return out
        y = conv_bn_act(self.conv1, self.bn1, xm, handoff=True)  # bn1's output feeds conv2 only
        return conv_bn_act(self.conv2, self.bn2, y, idt, dual=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, down=None):
        super().__init__()
        width = planes
        self.conv1 = _conv1x1(cin, width)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.conv2 = _conv3x3(width, width, stride)  # stride on the 3x3 (v1.5, as torchvision)
        self.bn2 = BatchNormAct2d(width, relu=True)
        self.conv3 = _conv1x1(width, planes * 4)
        self.bn3 = BatchNormAct2d(planes * 4, relu=True)  # relu(bn3(.) + identity), one fused op
        self.downsample = down

    def forward(self, x):
        # x: the previous block's output as (main, shortcut) aliases (bn_act dual=True: their
        # two gradients are summed inside the fused BN backward, not by an autograd add), or a
        # plain tensor for the first block
        xm, xs = x if isinstance(x, tuple) else (x, x)
        idt = xs if self.downsample is None else _down(self.downsample, xs)
        # the main path with bn1 / bn2 applied inside conv2 / conv3's GEMMs (ops/bnconv.py)
        out = bottleneck_main(self, xm, idt)
        if out is not None:
            return out
        # 1x1 conv -> BN pairs: the BN statistics may come from the conv GEMM's epilogue
        # (ops/conv.py conv_bn_act, autotuned; otherwise exactly bn(conv(x)))
        # bn1 / bn2 outputs feed exactly one conv each: their backward reductions come from the
        # consuming conv's data-grad GEMM epilogue (ops/bnact.py BNHandoff)
        y = conv_bn_act(self.conv1, self.bn1, xm, handoff=True)
        y = conv_bn_act(self.conv2, self.bn2, y, handoff=True)
        return conv_bn_act(self.conv3, self.bn3, y, idt, dual=True)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes=1000,
                 cifar_stem: bool = False):
        super().__init__()
        self.inplanes = 64
        if cifar_stem:
            self.conv1 = Conv2dSplitGrad(3, 64, 3, 1, 1, bias=False)
            self.maxpool = nn.Identity()
        else:
            self.conv1 = Conv2dSplitGrad(3, 64, 7, 2, 3, bias=False)
            self.maxpool = MaxPool2dNHWC(3, 2, 1)  # 1-byte window codes, gather backward
        self.bn1 = BatchNormAct2d(64, relu=True)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = GlobalAvgPoolFlat()  # mean over H, W + flatten; native broadcast backward
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, block, planes, n, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                                 BatchNormAct2d(planes * block.expansion))
        blocks = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        blocks += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*blocks)

    def forward(self, x):
        # stem: BN + ReLU + max pool fused (the BN output is never written; ops/bnact.py)
        # dual: the first block reads the pooled output twice (main path + shortcut); the two
        # gradients are summed inside the max-pool backward
        x = bn_relu_maxpool(self.conv1(x), self.bn1, self.maxpool, dual=True)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if isinstance(x, tuple):
            x = x[0]
        return self.fc(self.avgpool(x))


def resnet18(num_classes=1000):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes)


def resnet34(num_classes=1000):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes)


def resnet50(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes)


def resnet101(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes)


def resnet18_cifar(num_classes=10):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, cifar_stem=True)
