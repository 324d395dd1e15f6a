"""Perceiver building blocks with the reference's parameter layout.

The module tree exists for two reasons only: (1) it pins the ``state_dict``
key layout of the reference checkpoints and (2) it carries
an *eager* PyTorch forward that is the numerics oracle.  On an MI355X the
layer classes below (``CrossAttentionLayer`` / ``SelfAttentionLayer``) do not
walk their children at all: they hand their parameters to the fused HIP
executor in :mod:`perceiver_io_amd.ops.fused` (one autograd node per layer,
hand-written kernels for LN→QKV, attention, out-proj+residual+MLP).

Reference parity (behaviour, not code):
  * ``mlp``                       — ``perceiver/model.py:20-26`` (LN → Linear → GELU → Linear, width C→C→C)
  * ``cross_attention_layer``     — ``perceiver/model.py:29-33``
  * ``self_attention_layer/block``— ``perceiver/model.py:36-44``
  * ``Residual``                  — ``perceiver/model.py:47-56`` (residual on the first positional arg)
  * ``MultiHeadAttention``        — ``perceiver/model.py:59-74`` (nn.MultiheadAttention parameter names)
  * ``CrossAttention``            — ``perceiver/model.py:77-99`` (embed dim = num_q_channels)
  * ``SelfAttention``             — ``perceiver/model.py:102-116``
  * ``Sequential``                — ``perceiver/utils.py:7-14`` (tuple-splatting)
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class Sequential(nn.Sequential):
    """``nn.Sequential`` that splats a tuple result into the next module."""

    def forward(self, *inputs):
        for module in self:
            inputs = module(*inputs) if isinstance(inputs, tuple) else module(inputs)
        return inputs


def mlp(num_channels: int) -> Sequential:
    # children 0 (LN), 1 (Linear), 2 (GELU, no params), 3 (Linear) — key layout of App. C
    return Sequential(
        nn.LayerNorm(num_channels),
        nn.Linear(num_channels, num_channels),
        nn.GELU(),
        nn.Linear(num_channels, num_channels),
    )


class Residual(nn.Module):
    """``dropout(module(*args)) + args[0]``."""

    def __init__(self, module: nn.Module, dropout: float):
        super().__init__()
        self.module = module
        self.dropout = nn.Dropout(p=dropout)
        self.dropout_p = dropout

    def forward(self, *args, **kwargs):
        return self.dropout(self.module(*args, **kwargs)) + args[0]


class MHAParams(nn.Module):
    """Parameter container mirroring ``nn.MultiheadAttention``'s names and init.

    Keys: ``in_proj_weight`` (packed, when kdim == vdim == embed_dim) or
    ``q_proj_weight``/``k_proj_weight``/``v_proj_weight``; ``in_proj_bias``;
    ``out_proj.{weight,bias}``.  Init: xavier-uniform projections, zero biases,
    default ``nn.Linear`` init for the output projection weight.
    """

    def __init__(self, embed_dim: int, num_heads: int, kdim: int, vdim: int, dropout: float):
        super().__init__()
        if embed_dim % num_heads:
            raise ValueError(f"embed_dim {embed_dim} not divisible by num_heads {num_heads}")
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.kdim, self.vdim = kdim, vdim
        self.dropout = dropout
        self.batch_first = True
        self._qkv_same_embed_dim = kdim == embed_dim and vdim == embed_dim
        if self._qkv_same_embed_dim:
            self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
            self.register_parameter("q_proj_weight", None)
            self.register_parameter("k_proj_weight", None)
            self.register_parameter("v_proj_weight", None)
        else:
            self.q_proj_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
            self.k_proj_weight = nn.Parameter(torch.empty(embed_dim, kdim))
            self.v_proj_weight = nn.Parameter(torch.empty(embed_dim, vdim))
            self.register_parameter("in_proj_weight", None)
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim))
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        with torch.no_grad():
            if self._qkv_same_embed_dim:
                nn.init.xavier_uniform_(self.in_proj_weight)
            else:
                nn.init.xavier_uniform_(self.q_proj_weight)
                nn.init.xavier_uniform_(self.k_proj_weight)
                nn.init.xavier_uniform_(self.v_proj_weight)
            self.out_proj.bias.zero_()

    # -- views used by both backends -------------------------------------------------
    def q_weight(self):
        e = self.embed_dim
        return self.in_proj_weight[:e] if self._qkv_same_embed_dim else self.q_proj_weight

    def kv_weight(self):
        """(2E, kdim) packed K|V weight (a cat for the separate-weight layout)."""
        e = self.embed_dim
        if self._qkv_same_embed_dim:
            return self.in_proj_weight[e:]
        return torch.cat([self.k_proj_weight, self.v_proj_weight], 0)

    def qkv_weight(self):
        if self._qkv_same_embed_dim:
            return self.in_proj_weight
        return torch.cat([self.q_proj_weight, self.k_proj_weight, self.v_proj_weight], 0)


class MultiHeadAttention(nn.Module):
    def __init__(self, num_q_channels: int, num_kv_channels: int, num_heads: int, dropout: float):
        super().__init__()
        self.attention = MHAParams(num_q_channels, num_heads, num_kv_channels, num_kv_channels, dropout)

    def forward(self, x_q, x_kv, pad_mask=None, attn_mask=None):
        a = self.attention
        e = a.embed_dim
        if ops.get_backend() == "reference":
            # exactly nn.MultiheadAttention(batch_first=True).forward (need_weights=True)
            q, kv = x_q.transpose(0, 1), x_kv.transpose(0, 1)
            out, _ = F.multi_head_attention_forward(
                q, kv, kv, e, a.num_heads, a.in_proj_weight, a.in_proj_bias, None, None, False,
                a.dropout, a.out_proj.weight, a.out_proj.bias, training=self.training,
                key_padding_mask=pad_mask, need_weights=True, attn_mask=attn_mask,
                use_separate_proj_weight=not a._qkv_same_embed_dim, q_proj_weight=a.q_proj_weight,
                k_proj_weight=a.k_proj_weight, v_proj_weight=a.v_proj_weight)
            return out.transpose(0, 1)
        if x_q is x_kv and a._qkv_same_embed_dim:
            q, k, v = F.linear(x_q, a.in_proj_weight, a.in_proj_bias).split(e, dim=-1)
        else:
            q = F.linear(x_q, a.q_weight(), a.in_proj_bias[:e])
            k, v = F.linear(x_kv, a.kv_weight(), a.in_proj_bias[e:]).split(e, dim=-1)
        o = ops.attention.mha_core(q, k, v, a.num_heads, key_padding_mask=pad_mask, attn_mask=attn_mask,
                                   dropout_p=a.dropout if self.training else 0.0)
        return F.linear(o, a.out_proj.weight, a.out_proj.bias)


class CrossAttention(nn.Module):
    """LN on both streams, then MHA with embed dim = num_q_channels."""

    def __init__(self, num_q_channels: int, num_kv_channels: int, num_heads: int, dropout: float):
        super().__init__()
        self.q_norm = nn.LayerNorm(num_q_channels)
        self.kv_norm = nn.LayerNorm(num_kv_channels)
        self.attention = MultiHeadAttention(num_q_channels, num_kv_channels, num_heads, dropout)

    def forward(self, x_q, x_kv, pad_mask=None, attn_mask=None):
        return self.attention(self.q_norm(x_q), self.kv_norm(x_kv), pad_mask=pad_mask, attn_mask=attn_mask)


class SelfAttention(nn.Module):
    def __init__(self, num_channels: int, num_heads: int, dropout: float):
        super().__init__()
        self.norm = nn.LayerNorm(num_channels)
        self.attention = MultiHeadAttention(num_channels, num_channels, num_heads, dropout)

    def forward(self, x, pad_mask=None, attn_mask=None):
        x = self.norm(x)
        return self.attention(x, x, pad_mask=pad_mask, attn_mask=attn_mask)


class _FusedLayer(Sequential):
    """Residual(attention) → Residual(mlp) pair that can run as one fused node.

    Its parameters are flagged ``_pio_replicate``: a flat parameter space gives them 8-way
    replicated gradient accumulators, because every row tile of the fused backward adds its
    weight-gradient partial to them (ops/optim.py)."""

    def __init__(self, *modules):
        super().__init__(*modules)
        for p in self.parameters():
            p._pio_replicate = True

    @property
    def attn(self):
        return self[0].module

    @property
    def mlp(self):
        return self[1].module

    @property
    def dropout_p(self) -> float:
        return self[0].dropout_p

    def _fusable(self, x: torch.Tensor, attn_mask) -> bool:
        return attn_mask is None and ops.use_hip(x)

    def eager_forward(self, *args):
        return Sequential.forward(self, *args)


class CrossAttentionLayer(_FusedLayer):
    def forward(self, x_q, x_kv, pad_mask=None, attn_mask=None):
        if self._fusable(x_q, attn_mask):
            return ops.fused.cross_attention_layer(self, x_q, x_kv, pad_mask)
        return super().forward(x_q, x_kv, pad_mask, attn_mask)


class SelfAttentionLayer(_FusedLayer):
    def forward(self, x, pad_mask=None, attn_mask=None):
        if self._fusable(x, attn_mask) and pad_mask is None:
            return ops.fused.self_attention_layer(self, x)
        if pad_mask is None and attn_mask is None:
            return super().forward(x)
        return super().forward(x, pad_mask, attn_mask)


def cross_attention_layer(num_q_channels: int, num_kv_channels: int, num_heads: int, dropout: float):
    return CrossAttentionLayer(
        Residual(CrossAttention(num_q_channels, num_kv_channels, num_heads, dropout), dropout),
        Residual(mlp(num_q_channels), dropout),
    )


def self_attention_layer(num_channels: int, num_heads: int, dropout: float):
    return SelfAttentionLayer(
        Residual(SelfAttention(num_channels, num_heads, dropout), dropout),
        Residual(mlp(num_channels), dropout),
    )


def self_attention_block(num_layers: int, num_channels: int, num_heads: int, dropout: float):
    return Sequential(*[self_attention_layer(num_channels, num_heads, dropout) for _ in range(num_layers)])


def init_latent_(p: torch.Tensor) -> torch.Tensor:
    """N(0, 0.02) clamped to ±2 (``perceiver/model.py:169-174,222-227``)."""
    with torch.no_grad():
        return p.normal_(0.0, 0.02).clamp_(-2.0, 2.0)


__all__ = [
    "Sequential", "mlp", "Residual", "MHAParams", "MultiHeadAttention", "CrossAttention", "SelfAttention",
    "CrossAttentionLayer", "SelfAttentionLayer", "cross_attention_layer", "self_attention_layer",
    "self_attention_block", "init_latent_",
]
