"""ResNet-18/34/50/101/152 with torchvision-identical module and parameter names.

The reference trains ``torchvision.models.resnet18(pretrained=False)`` (1000-class
head kept even on CIFAR-10; cifar10-distributed-smddp-gpu.py:30-32) and saves
its DDP ``state_dict`` (keys ``module.conv1.weight`` ... ).  This
module reproduces that architecture (torchvision v1.5 layout: stride on the
3x3 conv of a Bottleneck) with the same names/shapes/buffers, so checkpoints
are interchangeable, while the CUDA forward/backward runs our fused kernels:
conv -> BN(+residual)(+ReLU) with the ReLU and residual add folded into the BN
apply kernel.
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

import os

from mi355x_dp.ops import resblock as _rb
from mi355x_dp.ops import stem as _stem
from .layers import BatchNorm2d, Conv2d, GlobalAvgPool2d, Linear, MaxPool2d, ReLU, conv_bn, to_device_input

# one fused autograd node per residual block on the native training path (MI355X_DP_FUSED_BLOCKS=0: per-op)
FUSED_BLOCKS = os.environ.get("MI355X_DP_FUSED_BLOCKS", "1") != "0"
# stem conv -> BN -> ReLU -> maxpool as one node (MI355X_DP_FUSED_STEM=0: per-op)
FUSED_STEM = os.environ.get("MI355X_DP_FUSED_STEM", "1") != "0"


def conv3x3(in_planes, out_planes, stride=1):
    return Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(in_planes, out_planes, stride=1):
    return Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if FUSED_BLOCKS and _rb.fusable(self, x):
            return _rb.res_block(self, x)
        identity = x
        out = conv_bn(self.conv1, self.bn1, x, relu=True)
        if self.downsample is not None:
            identity = conv_bn(self.downsample[0], self.downsample[1], x)
        return conv_bn(self.conv2, self.bn2, out, relu=True, residual=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = BatchNorm2d(planes * self.expansion)
        self.relu = ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if FUSED_BLOCKS and _rb.fusable(self, x):
            return _rb.res_block(self, x)
        identity = x
        out = conv_bn(self.conv1, self.bn1, x, relu=True)
        out = conv_bn(self.conv2, self.bn2, out, relu=True)
        if self.downsample is not None:
            identity = conv_bn(self.downsample[0], self.downsample[1], x)
        return conv_bn(self.conv3, self.bn3, out, relu=True, residual=identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNorm2d(self.inplanes)
        self.relu = ReLU(inplace=True)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = GlobalAvgPool2d()
        self.fc = Linear(512 * block.expansion, num_classes)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck) and m.bn3.weight is not None:
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock) and m.bn2.weight is not None:
                    nn.init.constant_(m.bn2.weight, 0)
        # checkpoints are written NCHW-contiguous regardless of the training layout
        self._register_state_dict_hook(_contiguous_state_dict_hook)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = to_device_input(x)
        if FUSED_STEM and _stem.fusable(self.conv1, self.bn1, self.maxpool, x):
            x = _stem.stem(self.conv1, self.bn1, self.maxpool, x)
        else:
            x = conv_bn(self.conv1, self.bn1, x, relu=True)
            x = self.maxpool(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        x = self.avgpool(x)
        return self.fc(x)


def _contiguous_state_dict_hook(module, state_dict, prefix, local_metadata):
    for k, v in list(state_dict.items()):
        if isinstance(v, torch.Tensor) and not v.is_contiguous():
            state_dict[k] = v.contiguous()
    return state_dict


def _resnet(block, layers, pretrained=False, progress=True, weights=None, **kwargs):
    if pretrained or weights is not None:
        raise RuntimeError("pretrained weights need network access; not available (random init only)")
    return ResNet(block, layers, **kwargs)


def resnet18(pretrained=False, progress=True, weights=None, **kwargs):
    return _resnet(BasicBlock, [2, 2, 2, 2], pretrained, progress, weights, **kwargs)


def resnet34(pretrained=False, progress=True, weights=None, **kwargs):
    return _resnet(BasicBlock, [3, 4, 6, 3], pretrained, progress, weights, **kwargs)


def resnet50(pretrained=False, progress=True, weights=None, **kwargs):
    return _resnet(Bottleneck, [3, 4, 6, 3], pretrained, progress, weights, **kwargs)


def resnet101(pretrained=False, progress=True, weights=None, **kwargs):
    return _resnet(Bottleneck, [3, 4, 23, 3], pretrained, progress, weights, **kwargs)


def resnet152(pretrained=False, progress=True, weights=None, **kwargs):
    return _resnet(Bottleneck, [3, 8, 36, 3], pretrained, progress, weights, **kwargs)
