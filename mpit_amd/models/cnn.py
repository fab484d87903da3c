"""Convolutional workloads other than ResNet.

* ``cnn7`` — the reference's CIFAR-10 7-layer CNN (asyncsgd/models/7-layers-cnn.lua:6-25):
  conv5(3→64)-ReLU-pool2, conv5(64→128)-ReLU-pool2, conv3(128→64)-ReLU, View(256),
  fc256-ReLU-Dropout(0.5), fc10, LogSoftMax; input 3×28×28; 351,946 parameters.
* ``lenet`` — LeNet-5 for MNIST (BASELINE.json config 1, the CPU/gloo plumbing run).
* ``alexnet`` — AlexNet (BASELINE.json config 4, Downpour with bounded staleness).
* ``vgg16`` — VGG-16 (BASELINE.json config 5, bf16 EASGD with bucket fusion).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.conv import ConvAct2d
from ..ops.linear import LinearAct
from ..ops.pool import MaxPool2dNHWC
from . import register


class CNN7(nn.Module):
    def __init__(self, num_classes: int = 10, dropout: float = 0.5):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 5), nn.ReLU(inplace=True), nn.MaxPool2d(2, 2),  # 28 -> 24 -> 12
            nn.Conv2d(64, 128, 5), nn.ReLU(inplace=True), nn.MaxPool2d(2, 2),  # 12 -> 8 -> 4
            nn.Conv2d(128, 64, 3), nn.ReLU(inplace=True),  # 4 -> 2 ; 64*2*2 = 256
        )
        self.classifier = nn.Sequential(
            nn.Linear(256, 256), nn.ReLU(inplace=True), nn.Dropout(dropout), nn.Linear(256, num_classes),
            nn.LogSoftmax(dim=1),
        )

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class LeNet(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(1, 6, 5, padding=2), nn.ReLU(inplace=True), nn.MaxPool2d(2),
            nn.Conv2d(6, 16, 5), nn.ReLU(inplace=True), nn.MaxPool2d(2),
        )
        self.classifier = nn.Sequential(
            nn.Linear(16 * 5 * 5, 120), nn.ReLU(inplace=True), nn.Linear(120, 84), nn.ReLU(inplace=True),
            nn.Linear(84, num_classes), nn.LogSoftmax(dim=1),
        )

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class AlexNet(nn.Module):
    """conv(+bias)+ReLU layers are :class:`ConvAct2d` (MFMA implicit GEMM with the bias and
    ReLU in the epilogue on MI355X; the 3-channel 11x11 stem stays on MIOpen) and the pools
    NHWC max-pool kernels."""

    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.features = nn.Sequential(
            ConvAct2d(3, 64, 11, stride=4, padding=2), MaxPool2dNHWC(3, 2),
            ConvAct2d(64, 192, 5, padding=2), MaxPool2dNHWC(3, 2),
            ConvAct2d(192, 384, 3, padding=1),
            ConvAct2d(384, 256, 3, padding=1),
            ConvAct2d(256, 256, 3, padding=1), MaxPool2dNHWC(3, 2),
        )
        self.avgpool = nn.AdaptiveAvgPool2d((6, 6))
        # Linear + ReLU pairs as LinearAct (ops/linear.py; the Identity keeps the reference's
        # layer indices, so state_dict keys are those of the nn.Linear / nn.ReLU layout)
        self.classifier = nn.Sequential(
            nn.Dropout(dropout), LinearAct(256 * 36, 4096), nn.Identity(),
            nn.Dropout(dropout), LinearAct(4096, 4096), nn.Identity(),
            LinearAct(4096, num_classes, act=False, pad_out=True),
        )

    def forward(self, x):
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


_VGG16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG(nn.Module):
    """Without batch norm every conv(+bias)+ReLU is one :class:`ConvAct2d` (bias and ReLU in
    the MFMA GEMM epilogue on MI355X; the 3-channel first layer on the row-tap kernel), the
    pools are NHWC max-pool kernels, and the classifier's Linear + ReLU pairs are
    :class:`LinearAct` (bf16 steps)."""

    def __init__(self, cfg=_VGG16, num_classes: int = 1000, dropout: float = 0.5, batch_norm: bool = False):
        super().__init__()
        layers, c = [], 3
        for v in cfg:
            if v == "M":
                layers.append(MaxPool2dNHWC(2, 2))
            elif batch_norm:
                layers += [nn.Conv2d(c, v, 3, padding=1), nn.BatchNorm2d(v), nn.ReLU(inplace=True)]
                c = v
            else:
                layers.append(ConvAct2d(c, v, 3, padding=1))
                c = v
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            LinearAct(512 * 49, 4096), nn.Identity(), nn.Dropout(dropout),
            LinearAct(4096, 4096), nn.Identity(), nn.Dropout(dropout),
            LinearAct(4096, num_classes, act=False, pad_out=True),
        )

    def forward(self, x):
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


@register("cnn7")
def cnn7(num_classes=10):
    return CNN7(num_classes)


@register("lenet")
def lenet(num_classes=10):
    return LeNet(num_classes)


@register("alexnet")
def alexnet(num_classes=1000):
    return AlexNet(num_classes)


@register("vgg16")
def vgg16(num_classes=1000):
    return VGG(_VGG16, num_classes)


INPUT_SHAPES = {
    "cnn7": (3, 28, 28),
    "lenet": (1, 28, 28),
    "alexnet": (3, 224, 224),
    "vgg16": (3, 224, 224),
    "resnet18": (3, 224, 224),
    "resnet34": (3, 224, 224),
    "resnet50": (3, 224, 224),
    "resnet101": (3, 224, 224),
    "resnet152": (3, 224, 224),
}
