"""ResNet (He et al. 2015, v1.5: stride on the 3x3 conv) — the BASELINE.json flagship
workload "ResNet-50 synthetic ImageNet". Written from the architecture definition
(torchvision is not available in this image); parameter count 25,557,032 for
ResNet-50 / 1000 classes, the standard figure.

Runs channels_last + bf16 autocast on MI355X: stride-1 1x1 convolutions on the
hand-written MFMA GEMMs, the 3x3s and strided 1x1 shortcuts on MFMA implicit GEMMs (strided
backward-data as parity classes), the 7x7 stem on the row-tap implicit GEMM
(mpit_amd/ops/conv.py), and every BatchNorm(+add)(+ReLU) on the fused HIP kernels
(ops/bn.py), whose statistics and backward reductions come from the GEMM epilogues.
"""
from __future__ import annotations

from typing import List, Type, Union

import os

import torch
import torch.nn as nn

from ..ops.bn import BatchNormAct2d, bn_pair
from ..ops.conv import Conv1x1, ConvNHWC, GradSlot, StemConv, feeds_bn, park_grad
from ..ops.linear import LinearAct
from ..ops.pool import GlobalAvgPoolNHWC, MaxPool2dNHWC

# Fused BN(+add)(+ReLU) HIP kernels on MI355X (mpit_amd/ops/bn.py); same parameters and
# state dict as nn.BatchNorm2d, and plain PyTorch math on CPU tensors.
FUSED_BN = True


def _bn(c, act):
    return BatchNormAct2d(c, act=act) if FUSED_BN else nn.BatchNorm2d(c)


def _feeds_bn(*pairs):
    """The MFMA convolutions whose outputs feed a fused BN emit its statistics from the GEMM
    accumulators and run that BN's forward finalize in their last blocks (ops/bn.py), so the
    BN forward is one apply pass. Each argument is a ``(conv, BN)`` pair, or a ``(conv, BN)``
    downsample Sequential as is."""
    for p in pairs:
        if p is None:
            continue
        if isinstance(p, nn.Sequential):
            if not (len(p) == 2 and isinstance(p[1], BatchNormAct2d)):
                continue
            p = (p[0], p[1])
        c, bn = p
        if FUSED_BN and hasattr(c, "emit_stats") and isinstance(bn, BatchNormAct2d):
            feeds_bn(c, bn)


# 1x1 convolutions as MFMA GEMMs and 3x3 ones as MFMA implicit GEMMs (both fall back to
# nn.Conv2d for CPU / odd shapes); MPIT_MFMA_CONV=0 routes them to MIOpen instead (A/B
# measurements), MPIT_MFMA_CONV3=0 only the 3x3s.
MFMA_CONV = os.environ.get("MPIT_MFMA_CONV", "1") != "0"
MFMA_CONV3 = MFMA_CONV and os.environ.get("MPIT_MFMA_CONV3", "1") != "0"
# MPIT_FC_FP32=1: the classifier runs in fp32 under bf16 autocast (round 4 default, when it was a
# hipBLASLt GEMM whose backward call left a host gap). Default: it follows autocast on LinearAct's
# bf16 MFMA path (fp32 accumulation, fp32 logits into the loss; its transpose is made by the
# step's weight cast launch) — no library GEMM in the step (tests/test_linear_act.py)
_FC_FP32 = os.environ.get("MPIT_FC_FP32", "0") != "0"


def conv3x3(i, o, stride=1):
    if MFMA_CONV3:
        return ConvNHWC(i, o, 3, stride=stride, padding=1)
    return nn.Conv2d(i, o, 3, stride=stride, padding=1, bias=False)


def conv1x1(i, o, stride=1):
    if MFMA_CONV:
        # strided (downsample) 1x1: implicit GEMM over the strided pixels (fwd, wgrad)
        return Conv1x1(i, o) if stride == 1 else ConvNHWC(i, o, 1, stride=stride)
    return nn.Conv2d(i, o, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inp, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inp, planes, stride)
        self.bn1 = _bn(planes, True)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _bn(planes, True)
        self.downsample = downsample
        _feeds_bn((self.conv1, self.bn1), (self.conv2, self.bn2), downsample)

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        if isinstance(self.bn1, BatchNormAct2d):
            out = self.bn1(self.conv1(x))
            return self.bn2(self.conv2(out), idt)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inp, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inp, planes)
        self.bn1 = _bn(planes, True)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = _bn(planes, True)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = _bn(planes * 4, True)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        _feeds_bn((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3), downsample)

    def forward(self, x):
        if isinstance(self.bn1, BatchNormAct2d):
            fused = (isinstance(self.conv1, Conv1x1) and self.conv1.fused(x) and self.bn3.fused(x)
                     and torch.is_grad_enabled())
            if fused and self.downsample is None:
                # identity shortcut: the shortcut gradient (dy*mask of bn3) is added inside
                # conv1's backward-data GEMM instead of by a separate autograd add
                slot = GradSlot()
                out = self.bn1(self.conv1(x, slot))
                out = self.bn2(self.conv2(out))
                return self.bn3(self.conv3(out), x, res_slot=slot)
            if fused:
                # downsample shortcut, computed after the main branch so that its backward runs
                # first: the shortcut conv's input gradient is parked and added in conv1's
                # backward-data epilogue (no autograd add over the block input)
                slot = GradSlot()
                out = self.bn1(self.conv1(x, slot))
                out = self.bn2(self.conv2(out))
                out = self.conv3(out)
                conv_ds, bn_ds = self.downsample[0], self.downsample[1]
                if isinstance(bn_ds, BatchNormAct2d) and len(self.downsample) == 2:
                    # relu(bn3(out) + bn_ds(conv_ds(x))) as one op: no shortcut tensor, one
                    # pass each way for both BNs (ops/bn.py bn_pair)
                    return bn_pair(self.bn3, out, bn_ds, conv_ds(park_grad(x, slot)))
                idt = self.downsample(park_grad(x, slot))
                return self.bn3(out, idt)
            idt = x if self.downsample is None else self.downsample(x)
            out = self.bn1(self.conv1(x))
            out = self.bn2(self.conv2(out))
            return self.bn3(self.conv3(out), idt)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        # 7x7 stem on the MFMA row-tap kernels (ops/conv.py StemConv), emitting bn1's statistics
        self.conv1 = StemConv(3, 64, 7, 2, 3) if MFMA_CONV else nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64, True)
        _feeds_bn((self.conv1, self.bn1))
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool2dNHWC(3, stride=2, padding=1) if MFMA_CONV else nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = GlobalAvgPoolNHWC() if MFMA_CONV else nn.AdaptiveAvgPool2d(1)
        # the classifier on the MFMA kernels in bf16 steps (ops/linear.py; N padded to 64 inside
        # the GEMMs): no hipBLASLt call and no per-step weight / gradient casts. nn.Linear's
        # parameters and state_dict keys; fp32 steps run F.linear
        self.fc = (LinearAct(512 * block.expansion, num_classes, act=False, pad_out=True) if MFMA_CONV
                   else nn.Linear(512 * block.expansion, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes BatchNormAct2d
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)
        self._plan_planes()

    def _plan_planes(self):
        """fp32 steps: which tensors are written as fp16 planes (ops/conv.py _F32_PLANES) —
        every activation and gradient that only GEMMs (and the residual adds, which decode them)
        read: the stem pool's output, each block's BN outputs and its BNs' input gradients. Not
        the stem BN's (it feeds the pool; its gradient feeds the row-tap stem wgrad), and not at
        the end of the network: the last block's output feeds the average pool, its last BN's
        gradient comes from that pool (no producing GEMM to know its max), so the last
        convolution's input and gradient stay fp32 (a backward-weight GEMM takes both operands
        as planes or neither)."""
        if not isinstance(self.bn1, BatchNormAct2d) or not isinstance(self.maxpool, MaxPool2dNHWC):
            return
        self.maxpool.out_planes = True
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        for b in blocks:
            bns = [b.bn1, b.bn2] + ([b.bn3] if isinstance(b, Bottleneck) else [])
            if b.downsample is not None and len(b.downsample) == 2:
                bns.append(b.downsample[1])
            for bn in bns:
                if isinstance(bn, BatchNormAct2d):
                    bn.out_planes = bn.grad_planes = True
        last = blocks[-1]
        feed_last, out_last = (last.bn2, last.bn3) if isinstance(last, Bottleneck) else (last.bn1, last.bn2)
        feed_last.out_planes = False
        out_last.out_planes = out_last.grad_planes = False

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 _bn(planes * block.expansion, False))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        if isinstance(self.bn1, BatchNormAct2d):
            x = self.maxpool(self.bn1(self.conv1(x)))
        else:
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        if _FC_FP32 and x.is_cuda and torch.is_autocast_enabled("cuda"):
            # (MPIT_FC_FP32=1) the classifier in fp32 under bf16 autocast, on LinearAct's fp32
            # path (its own transpose per call: the step's cast launch is bf16)
            with torch.autocast("cuda", enabled=False):
                return self.fc(x.float())
        return self.fc(x)


def resnet18(num_classes=1000):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes)


def resnet34(num_classes=1000):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes)


def resnet50(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes)


def resnet101(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes)


def resnet152(num_classes=1000):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes)
