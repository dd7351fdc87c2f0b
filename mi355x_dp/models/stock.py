"""The same torchvision-compatible ResNet built from STOCK torch.nn layers
(MIOpen / rocBLAS / ATen on the GPU).  Used as the comparison point for
numerics (tests) and for the stock-PyTorch throughput baseline (tools/)."""
import importlib

import torch
import torch.nn as nn
import torch.nn.functional as F


class StockBN(nn.BatchNorm2d):
    def forward(self, x, relu=False, residual=None):
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y


class StockGAP(nn.AdaptiveAvgPool2d):
    def __init__(self):
        super().__init__((1, 1))

    def forward(self, x):
        return torch.flatten(super().forward(x), 1)


def stock_resnet(name: str, num_classes: int = 1000):
    """Fresh module namespace so the patched layer classes never leak into mi355x_dp.models."""
    spec = importlib.util.find_spec("mi355x_dp.models.resnet")
    R = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(R)
    R.Conv2d, R.BatchNorm2d, R.Linear, R.MaxPool2d, R.GlobalAvgPool2d = (
        nn.Conv2d, StockBN, nn.Linear, nn.MaxPool2d, StockGAP)
    R.to_device_input = lambda x: x
    R.conv_bn = lambda conv, bn, x, relu=False, residual=None: bn(conv(x), relu=relu, residual=residual)
    return getattr(R, name)(num_classes=num_classes)
