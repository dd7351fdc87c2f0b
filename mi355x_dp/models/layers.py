"""nn.Module layers whose CUDA forward runs the native gfx950 kernels.

Each class subclasses the matching ``torch.nn`` module, so parameter/buffer
names, ``state_dict`` layout, ``repr`` and ``isinstance`` checks are identical
to stock PyTorch / torchvision (checkpoint compatibility).
On host tensors they run the stock fp32 PyTorch math.  With ``MI355X_DP_COMPUTE_DTYPE=fp32``
(``mi355x_dp.ops.fp32``) CUDA activations stay fp32 and every layer runs the native fp32 kernels
(shapes they do not cover fall back to stock fp32 PyTorch).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from mi355x_dp.ops import fp32 as F32m
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
        if F32m.active(x):
            if (self.groups == 1 and self.padding_mode == "zeros" and not isinstance(self.padding, str)
                    and _pair_square(self.dilation, "dilation") == 1 and self.out_channels % 4 == 0):
                return F32m.conv2d(x, self.weight, self.bias, _pair_square(self.stride, "stride"),
                                   _pair_square(self.padding, "padding"))
            return super().forward(x[:, :self.in_channels] if x.shape[1] != self.in_channels else x)
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
        if F32m.active(x) and x.shape[1] % 4 == 0:
            return F32m.batch_norm_act(x, self.weight, self.bias,
                                       self.running_mean if self.track_running_stats else None,
                                       self.running_var if self.track_running_stats else None,
                                       self.num_batches_tracked if (self.training and self.track_running_stats)
                                       else None, use_batch, eaf, self.eps, relu, residual)
        if F32m.active(x):  # a channel count the fp32 kernels do not cover: stock fp32 math
            y = F.batch_norm(x, self.running_mean if (not self.training or self.track_running_stats) else None,
                             self.running_var if (not self.training or self.track_running_stats) else None,
                             self.weight, self.bias, use_batch, eaf, self.eps)
            if self.training and self.track_running_stats and self.num_batches_tracked is not None:
                self.num_batches_tracked.add_(1)
            y = y + residual if residual is not None else y
            return F.relu(y) if relu else y
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
        if F32m.active(x):
            if self.in_features % 4 == 0 and self.out_features % 4 == 0:
                return F32m.linear(x, self.weight, self.bias)
            return F.linear(x, self.weight, self.bias)
        if not x.is_cuda:
            return super().forward(x.float() if x.dtype != self.weight.dtype else x)
        return Fm.linear(x, self.weight, self.bias)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x)
        if self.dilation not in (1, (1, 1)) or self.ceil_mode:
            if F32m.active(x):
                return super().forward(x)
            raise NotImplementedError("native maxpool: dilation=1, ceil_mode=False")
        if F32m.active(x):
            return F32m.max_pool2d(x, _pair_square(self.kernel_size, "kernel"), _pair_square(self.stride, "stride"),
                                   _pair_square(self.padding, "padding"))
        return Fm.max_pool2d(x, _pair_square(self.kernel_size, "kernel"), _pair_square(self.stride, "stride"),
                             _pair_square(self.padding, "padding"))


class GlobalAvgPool2d(nn.AdaptiveAvgPool2d):
    """AdaptiveAvgPool2d((1, 1)) followed by flatten(1) -> [N, C]."""

    def __init__(self):
        super().__init__((1, 1))

    def forward(self, x):
        if F32m.active(x):
            return F32m.global_avg_pool(x)
        return Fm.global_avg_pool(x)


class ReLU(nn.ReLU):
    pass


def conv_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool = False, residual=None):
    """act(bn(conv(x)) + residual).  On the native training path the conv epilogue also emits the
    BN batch-statistics partials, so BN never re-reads the conv output to compute them."""
    if (x.is_cuda and bn.training and isinstance(conv, Conv2d) and isinstance(bn, BatchNorm2d)
            and conv.bias is None and conv.groups == 1 and not F32m.active(x)):
        y, st = Fm.conv2d_with_stats(x, conv.weight, _pair_square(conv.stride, "stride"),
                                     _pair_square(conv.padding, "padding"))
        return bn(y, relu=relu, residual=residual, stats=st)
    return bn(conv(x), relu=relu, residual=residual)


def to_device_input(x: torch.Tensor) -> torch.Tensor:
    """Model-entry conversion for the native path: bf16, NHWC storage; images with <= 8 channels are
    zero-padded to 8 (one 16-byte chunk per pixel, the stem conv's gather unit).  fp32 compute mode:
    fp32 NHWC, channels zero-padded to a multiple of 4."""
    if x.is_cuda and F32m.COMPUTE_FP32:
        return F32m.to_input(x)
    if x.is_cuda:
        if x.dim() == 4 and x.shape[1] < 8:
            return Fm.pad_channels8(x)
        return x.to(dtype=torch.bfloat16, memory_format=torch.channels_last)
    return x
