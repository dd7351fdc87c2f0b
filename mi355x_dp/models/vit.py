"""ViT-B/16 with torchvision-identical module / parameter names (BASELINE.json config 5:
"ViT-B/16 bf16 DDP ... pure-GEMM MFMA path, same DDP engine"; SURVEY.md §2.5 note).

    conv_proj, class_token, encoder.pos_embedding,
    encoder.layers.encoder_layer_{i}.{ln_1, self_attention.{in_proj_weight, in_proj_bias,
    out_proj.weight, out_proj.bias}, ln_2, mlp.{0,3}.{weight,bias}}, encoder.ln, heads.head

(86,567,656 parameters for B/16 @ 224, 1000 classes.)  On the GPU every GEMM -- patch
embedding (as a stride-16 implicit-GEMM conv, small-channel mode), the fused QKV
projection, attention output projection, both MLP projections and the head -- runs on
the MFMA kernels in bf16 with fp32 master weights in the flat DP engine.  On the GPU each
encoder block is one fused autograd node (``mi355x_dp.ops.transformer.encoder_layer``):
native LayerNorm kernels, GELU and residual adds in the GEMM epilogues, bias gradients as
bf16 column sums.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from mi355x_dp.ops import functional as Fm
from mi355x_dp.ops import transformer as Tm
from .layers import Conv2d, Linear


# MI355X_DP_VIT_EMBED=0: the stock concatenation / broadcast add / full-sequence final LayerNorm (A/B)
_NATIVE_EMBED = os.environ.get("MI355X_DP_VIT_EMBED", "1") != "0"


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose fp32 (master) affine params follow a bf16 activation's dtype."""

    def forward(self, x):
        if x.is_cuda and self.elementwise_affine and self.weight.dtype == torch.float32:
            return Tm.layer_norm(x, self.weight, self.bias, self.eps)
        w = self.weight.to(x.dtype) if self.weight is not None else None
        b = self.bias.to(x.dtype) if self.bias is not None else None
        return F.layer_norm(x, self.normalized_shape, w, b, self.eps)


class MultiheadSelfAttention(nn.Module):
    """Parameter layout of nn.MultiheadAttention(embed_dim, num_heads, batch_first=True)."""

    def __init__(self, dim, heads, dropout=0.0):
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout = dim, heads, dropout
        self.head_dim = dim // heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * dim, dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * dim))
        self.out_proj = nn.Linear(dim, dim)  # NonDynamicallyQuantizableLinear in torch; same params
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, x):
        B, T, D = x.shape
        if x.is_cuda:
            qkv = Fm.linear(x, self.in_proj_weight, self.in_proj_bias, out_bf16=True)
        else:
            qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias)
        q, k, v = qkv.view(B, T, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4).unbind(0)
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0)
        o = o.transpose(1, 2).reshape(B, T, D)
        if x.is_cuda:
            return Fm.linear(o, self.out_proj.weight, self.out_proj.bias, out_bf16=True)
        return self.out_proj(o)


class MLPBlock(nn.Sequential):
    def __init__(self, dim, mlp_dim, dropout=0.0):
        super().__init__(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Dropout(dropout), nn.Linear(mlp_dim, dim),
                         nn.Dropout(dropout))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)

    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x)
        h = Fm.linear(x, self[0].weight, self[0].bias, out_bf16=True)
        h = self[2](F.gelu(h))
        return self[4](Fm.linear(h, self[3].weight, self[3].bias, out_bf16=True))


class EncoderBlock(nn.Module):
    def __init__(self, heads, dim, mlp_dim, dropout=0.0, attention_dropout=0.0):
        super().__init__()
        self.num_heads = heads
        self.ln_1 = LayerNorm(dim, eps=1e-6)
        self.self_attention = MultiheadSelfAttention(dim, heads, attention_dropout)
        self.dropout = nn.Dropout(dropout)
        self.ln_2 = LayerNorm(dim, eps=1e-6)
        self.mlp = MLPBlock(dim, mlp_dim, dropout)

    def fused_params(self):
        return [self.get_parameter(n) for n in Tm.PARAM_ORDER]

    def forward(self, x):
        fusable = (self.self_attention.dropout == 0.0 and self.dropout.p == 0.0 and self.mlp[2].p == 0.0) \
            or not self.training
        if x.is_cuda and fusable and self.ln_1.weight.dtype == torch.float32:
            return Tm.encoder_layer(x, self.num_heads, self.ln_1.eps, self.fused_params())
        y = self.dropout(self.self_attention(self.ln_1(x))) + x
        return self.mlp(self.ln_2(y)) + y


class Encoder(nn.Module):
    def __init__(self, seq_length, num_layers, heads, dim, mlp_dim, dropout=0.0, attention_dropout=0.0):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_length, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(dropout)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim, dropout, attention_dropout))
            for i in range(num_layers)))
        self.ln = LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        x = x + self.pos_embedding.to(x.dtype)
        return self.ln(self.layers(self.dropout(x)))


class VisionTransformer(nn.Module):
    def __init__(self, image_size=224, patch_size=16, num_layers=12, num_heads=12, hidden_dim=768, mlp_dim=3072,
                 dropout=0.0, attention_dropout=0.0, num_classes=1000):
        super().__init__()
        self.image_size, self.patch_size, self.hidden_dim = image_size, patch_size, hidden_dim
        self.num_classes = num_classes
        self.conv_proj = Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        seq = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.encoder = Encoder(seq, num_layers, num_heads, hidden_dim, mlp_dim, dropout, attention_dropout)
        self.seq_length = seq
        self.heads = nn.Sequential(OrderedDict(head=Linear(hidden_dim, num_classes)))
        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    def _process_input(self, x):
        n = x.shape[0]
        if _NATIVE_EMBED and Tm.patch_embed_ok(x, self.conv_proj):
            return Tm.patch_embed(x, self.conv_proj)  # patchify + one plain GEMM: [N, h*w, D]
        x = self.conv_proj(x)                 # [N, D, h, w]  (channels_last on the GPU path)
        x = x.permute(0, 2, 3, 1).reshape(n, -1, self.hidden_dim)  # NHWC storage: a free view
        return x

    def forward(self, x):
        if x.is_cuda:
            if x.shape[1] < 8:
                x = Fm.pad_channels8(x)
            else:
                x = x.to(torch.bfloat16, memory_format=torch.channels_last)
        x = self._process_input(x)
        n = x.shape[0]
        if x.is_cuda and _NATIVE_EMBED and x.dtype == torch.bfloat16 and self.class_token.dtype == torch.float32 \
                and self.hidden_dim % 8 == 0:
            # class token + position embedding in one native pass (ops.transformer.vit_embed); the
            # head reads only the class token and LayerNorm is per token, so the final LayerNorm
            # runs on those rows alone -- the same output as encoder(x)[:, 0]
            enc = self.encoder
            x = enc.layers(enc.dropout(Tm.vit_embed(x, self.class_token, enc.pos_embedding)))
            return self.heads(enc.ln(x[:, 0]))
        x = torch.cat([self.class_token.expand(n, -1, -1).to(x.dtype), x], dim=1)
        x = self.encoder(x)
        return self.heads(x[:, 0])


def vit_b_16(num_classes=1000, image_size=224, **kw):
    return VisionTransformer(image_size=image_size, patch_size=16, num_layers=12, num_heads=12, hidden_dim=768,
                             mlp_dim=3072, num_classes=num_classes, **kw)
