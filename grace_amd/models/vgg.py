"""VGG-16 (Simonyan & Zisserman, 2015) -- BASELINE config 3 (PowerSGD rank-4).

torchvision layout ``vgg16``: 13 3x3 convs (64,64,M,128,128,M,256x3,M,512x3,M,512x3,M),
adaptive 7x7 pool, classifier 25088-4096-4096-1000 with dropout; 138,357,544 parameters.
fc6 (4096 x 25088 = 103M) is the tall-skinny PowerSGD stress case.
"""
import torch
import torch.nn as nn

from ..ops.convact import ConvBiasAct2d
from ..ops.pool import MaxPool2dNHWC

_CFG16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG(nn.Module):
    def __init__(self, cfg=_CFG16, num_classes=1000, batch_norm=False):
        super().__init__()
        layers, c = [], 3
        for v in cfg:
            if v == "M":
                layers.append(MaxPool2dNHWC(2, 2))
            elif batch_norm:
                layers += [nn.Conv2d(c, v, 3, padding=1), nn.BatchNorm2d(v), nn.ReLU(inplace=True)]
                c = v
            else:
                # conv + bias + ReLU with the bias add and ReLU as native kernels (ops/convact.py);
                # the Identity keeps torchvision's features.<i> indices / state_dict keys
                layers += [ConvBiasAct2d(c, v, 3, padding=1, relu=True), nn.Identity()]
                c = v
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


def vgg16(num_classes=1000):
    return VGG(_CFG16, num_classes)
