"""nn.Module layers whose CUDA forward runs the native gfx950 kernels.

Each class subclasses the matching ``torch.nn`` module, so parameter/buffer
names, ``state_dict`` layout, ``repr`` and ``isinstance`` checks are identical
to stock PyTorch / torchvision (checkpoint compatibility).
On host tensors they run the stock fp32 PyTorch math.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from mi355x_dp.ops import functional as Fm


def _pair_square(v, what):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise NotImplementedError(f"non-square {what} {v} on the native path")
        return int(v[0])
    return int(v)


class Conv2d(nn.Conv2d):
    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x)
        if self.groups != 1 or _pair_square(self.dilation, "dilation") != 1 or self.padding_mode != "zeros":
            raise NotImplementedError("native conv supports groups=1, dilation=1, zero padding")
        if isinstance(self.padding, str):
            raise NotImplementedError("string padding on the native path")
        return Fm.conv2d(x, self.weight, self.bias, _pair_square(self.stride, "stride"),
                         _pair_square(self.padding, "padding"))


class BatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d with optional fused residual add and ReLU: ``act(bn(x) + residual)``."""

    def forward(self, x, relu: bool = False, residual=None, stats=None):
        if self.momentum is None:
            eaf = 0.0
        else:
            eaf = self.momentum
        use_batch = self.training or (self.running_mean is None)
        if self.training and self.track_running_stats and self.momentum is None and self.num_batches_tracked is not None:
            eaf = 1.0 / float(self.num_batches_tracked.item() + 1)
        if not x.is_cuda:
            return Fm.batch_norm_act(x, self.weight, self.bias,
                                     self.running_mean if (not self.training or self.track_running_stats) else None,
                                     self.running_var if (not self.training or self.track_running_stats) else None,
                                     self.num_batches_tracked if self.training and self.track_running_stats else None,
                                     use_batch, eaf, self.eps, relu, residual)
        return Fm.batch_norm_act(x, self.weight, self.bias,
                                 self.running_mean if self.track_running_stats else None,
                                 self.running_var if self.track_running_stats else None,
                                 self.num_batches_tracked if (self.training and self.track_running_stats) else None,
                                 use_batch, eaf, self.eps, relu, residual, stats if use_batch else None)


class Linear(nn.Linear):
    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x.float() if x.dtype != self.weight.dtype else x)
        return Fm.linear(x, self.weight, self.bias)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x)
        if self.dilation not in (1, (1, 1)) or self.ceil_mode:
            raise NotImplementedError("native maxpool: dilation=1, ceil_mode=False")
        return Fm.max_pool2d(x, _pair_square(self.kernel_size, "kernel"), _pair_square(self.stride, "stride"),
                             _pair_square(self.padding, "padding"))


class GlobalAvgPool2d(nn.AdaptiveAvgPool2d):
    """AdaptiveAvgPool2d((1, 1)) followed by flatten(1) -> [N, C]."""

    def __init__(self):
        super().__init__((1, 1))

    def forward(self, x):
        return Fm.global_avg_pool(x)


class ReLU(nn.ReLU):
    pass


def conv_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool = False, residual=None):
    """act(bn(conv(x)) + residual).  On the native training path the conv epilogue also emits the
    BN batch-statistics partials, so BN never re-reads the conv output to compute them."""
    if (x.is_cuda and bn.training and isinstance(conv, Conv2d) and isinstance(bn, BatchNorm2d)
            and conv.bias is None and conv.groups == 1):
        y, st = Fm.conv2d_with_stats(x, conv.weight, _pair_square(conv.stride, "stride"),
                                     _pair_square(conv.padding, "padding"))
        return bn(y, relu=relu, residual=residual, stats=st)
    return bn(conv(x), relu=relu, residual=residual)


def to_device_input(x: torch.Tensor) -> torch.Tensor:
    """Model-entry conversion for the native path: bf16, NHWC storage; images with <= 8 channels are
    zero-padded to 8 (one 16-byte chunk per pixel, the stem conv's gather unit)."""
    if x.is_cuda:
        if x.dim() == 4 and x.shape[1] < 8:
            return Fm.pad_channels8(x)
        return x.to(dtype=torch.bfloat16, memory_format=torch.channels_last)
    return x
