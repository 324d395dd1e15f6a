"""Context (sequence) parallelism for the Perceiver encoder (stretch goal).

The reference has no sequence parallelism: every rank holds the whole input and the encoder
cross-attention reads all M keys (``perceiver/model.py:150-160,185-187``).  The Perceiver
makes a cheap context-parallel scheme possible that ring attention is not needed for: the
inputs are only ever the keys/values of a cross-attention from N ≪ M latents, so

  * each rank of a CP group holds a contiguous slice of the M inputs (its shard of the input
    adapter output, LayerNorm and K/V projection: the dominant cost at long M);
  * per cross-attention it computes its partial softmax state for the replicated latent
    queries — un-normalised ``O_r = Σ_k exp(s - m) V`` and ``l_r = Σ_k exp(s - m)`` with a
    group-wide max ``m`` (one all-reduce MAX of B·h·N floats);
  * one all-reduce SUM of ``[O_r ‖ l_r]`` (B·h·N·(d+1) floats, ≈ N·C per sample — tiny next to
    the K/V shard) combines them; ``O / l`` is the exact attention output;
  * everything after (out-projection, MLP, the latent self-attention stack, the decoder) runs
    replicated on the latents.

Gradients (Megatron-style conjugate pairs, one per cross-attention):
  * combine: all-reduce SUM forward, identity backward (each rank's partial gets the common
    upstream gradient);
  * the replicated queries enter the shard-local score computation through an identity whose
    backward all-reduces (SUM) the query gradient — every replicated activation and parameter
    upstream then sees the full, identical gradient on all ranks;
  * the shard-local K/V (after the projection) pass ``world_cp × grad`` backward, so after the
    usual data-parallel *average* over the whole world (``FlatGradReducer``) the shard-local
    parameters (input adapter, kv LayerNorm, K/V projection) hold the sum of their shard
    contributions — exact full-sequence gradients, no change to the reducer.
Fully masked rows (every key of every shard PAD) give 0, as in the single-GPU kernels
(defect D10).

On a GPU the shard-local attention runs on the flash-attention kernels (``csrc/attention.hip``,
no score matrix in memory): the forward kernel returns the shard's normalised output and its
log-sum-exp; the ranks merge them with one all-reduce MAX of the LSE and one all-reduce SUM of
``[w_r·O_r ‖ w_r]`` (``w_r = 2^(lse_r − max)``), which also gives the global LSE.  The backward
kernel, fed the GLOBAL output and LSE, yields this shard's exact dK/dV and a partial dQ (summed
by the replicated-input identity).  ``impl="torch"`` (the CPU default) keeps the plain fp32
PyTorch math.  Dropout must be 0 (replicated computations would otherwise draw different masks
per rank).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def _group_size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _group_rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def shard_range(m: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous near-equal split of ``m`` inputs: rank r gets ``[lo, hi)``."""
    base, rem = divmod(m, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


class _SumCombine(torch.autograd.Function):
    """All-reduce SUM of per-shard partials; identity backward."""

    @staticmethod
    def forward(ctx, t, group):
        out = t.clone()
        if _group_size(group) > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, None


class _ReplicatedIn(torch.autograd.Function):
    """Identity forward; backward all-reduces (SUM) the gradient of a replicated tensor that
    feeds shard-local work."""

    @staticmethod
    def forward(ctx, t, group):
        ctx.group = group
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        if _group_size(ctx.group) > 1:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
        return g, None


class _ShardGradScale(torch.autograd.Function):
    """Identity forward; backward multiplies by the group size (shard-local gradients are
    later averaged over the world, see module doc)."""

    @staticmethod
    def forward(ctx, t, world):
        ctx.world = world
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.world, None


class _ShardFlashAttention(torch.autograd.Function):
    """Shard-local flash attention merged over ``group`` (module doc): q (B, N, E) replicated,
    k / v (B, M_local, E) this rank's keys → the exact full-sequence output (B, N, E) fp32."""

    @staticmethod
    def forward(ctx, q, k, v, kmask, H, D, scale, group):
        from ..ops.fused import kernels

        K = kernels(q)
        B, N, E = q.shape
        qb, kb, vb = (t.to(torch.bfloat16).contiguous() for t in (q, k, v))
        km = kmask.to(torch.bool).contiguous() if kmask is not None else None
        if k.shape[1] > 0:
            o_r, l2 = K.attn_fwd(qb, kb, vb, km, H, D, scale, 0.0, None, 1)  # lse in log2 units, +inf: no key
            l2 = torch.where(torch.isfinite(l2), l2, torch.full_like(l2, float("-inf")))
            o_r = o_r.float().view(B, N, H, D)
        else:  # an empty shard contributes nothing
            l2 = torch.full((B, N, H), float("-inf"), device=q.device)
            o_r = torch.zeros((B, N, H, D), device=q.device)
        m = l2.clone()
        if _group_size(group) > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
        w = torch.exp2(l2 - m)  # (B, N, H); 0 for a shard without live keys
        packed = torch.cat([o_r * w[..., None], w[..., None]], dim=-1)
        if _group_size(group) > 1:
            dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
        S = packed[..., D]
        o = torch.where(S[..., None] > 0, packed[..., :D] / S.clamp_min(1e-30)[..., None], torch.zeros_like(o_r))
        lse = torch.where(S > 0, m + torch.log2(S.clamp_min(1e-30)), torch.full_like(S, float("inf")))
        o = o.reshape(B, N, E)
        ob = o.to(torch.bfloat16).contiguous()
        ctx.save_for_backward(qb, kb, vb, ob, lse.contiguous(), km if km is not None else torch.empty(0))
        ctx.cfg = (H, D, scale, km is not None)
        return o

    @staticmethod
    def backward(ctx, g):
        from ..ops.fused import kernels

        qb, kb, vb, ob, lse, km = ctx.saved_tensors
        H, D, scale, has_mask = ctx.cfg
        if kb.shape[1] == 0:
            return torch.zeros_like(g), torch.zeros(kb.shape, device=g.device), torch.zeros(vb.shape, device=g.device), \
                None, None, None, None, None
        dq, dk, dv = kernels(g).attn_bwd(qb, kb, vb, km if has_mask else None, ob, g.to(torch.bfloat16).contiguous(), lse,
                                         None, H, D, scale, 0.0, None, None, None, None)
        return dq, dk, dv, None, None, None, None, None


def _default_impl(t: torch.Tensor) -> str:
    from .. import ops

    return "kernel" if ops.use_hip(t) else "torch"


def cp_cross_attention(attn, x_q: torch.Tensor, x_kv: torch.Tensor, pad_mask: Optional[torch.Tensor], group=None,
                       impl: Optional[str] = None):
    """``CrossAttention`` (q_norm / kv_norm / MHA, ``perceiver/model.py:77-99``) over this
    rank's K/V shard, combined over ``group`` into the exact full-sequence output.
    ``impl``: "kernel" (flash-attention kernels; the default on a GPU) or "torch"."""
    a = attn.attention.attention  # MHAParams (nn.MultiheadAttention layout)
    e, h = a.embed_dim, a.num_heads
    d = e // h
    world = _group_size(group)
    q = _ReplicatedIn.apply(F.linear(attn.q_norm(x_q), a.q_weight(), a.in_proj_bias[:e]), group)
    kv = _ShardGradScale.apply(F.linear(attn.kv_norm(x_kv), a.kv_weight(), a.in_proj_bias[e:]), world)
    k, v = kv.split(e, dim=-1)
    if (impl or _default_impl(x_q)) == "kernel" and d in (16, 32, 64, 128):
        qc = q.contiguous() if q.stride(-1) == 1 and q.shape[0] == k.shape[0] else q.expand(k.shape[0], -1, -1).contiguous()
        o = _ShardFlashAttention.apply(qc, k, v, pad_mask, h, d, 1.0 / math.sqrt(d), group)
        return F.linear(o.to(x_q.dtype), a.out_proj.weight, a.out_proj.bias)
    B, N, _ = q.shape
    M = k.shape[1]
    q = q.view(B, N, h, d).transpose(1, 2) * (1.0 / math.sqrt(d))
    k = k.view(B, M, h, d).transpose(1, 2)
    v = v.view(B, M, h, d).transpose(1, 2)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2))  # (B, h, N, M_local)
    if pad_mask is not None:
        s = s.masked_fill(pad_mask[:, None, None, :].to(torch.bool), float("-inf"))
    with torch.no_grad():  # the max is only a shift: it cancels in O / l
        m = s.amax(dim=-1, keepdim=True) if M > 0 else torch.full((B, h, N, 1), float("-inf"), device=s.device)
        if _group_size(group) > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    p = torch.exp(s - m)  # masked keys → exp(-inf) = 0
    o = torch.matmul(p, v.float())
    packed = _SumCombine.apply(torch.cat([o, p.sum(dim=-1, keepdim=True)], dim=-1), group)
    o, l = packed[..., :d], packed[..., d:]
    o = torch.where(l > 0, o / l.clamp_min(1e-30), torch.zeros_like(o))  # fully masked rows → 0 (D10)
    o = o.transpose(1, 2).reshape(B, N, e).to(x_q.dtype)
    return F.linear(o, a.out_proj.weight, a.out_proj.bias)


def cp_cross_attention_layer(layer, x_q, x_kv, pad_mask, group=None, impl=None):
    """``Residual(CrossAttention)`` then ``Residual(mlp)`` (``perceiver/model.py:29-33``)."""
    att_res, mlp_res = layer[0], layer[1]
    y = att_res.dropout(cp_cross_attention(att_res.module, x_q, x_kv, pad_mask, group, impl)) + x_q
    return mlp_res.dropout(mlp_res.module(y)) + y


def shard_input(adapter, x: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    """The input adapter's output restricted to inputs ``[lo, hi)`` without computing the rest
    (text: embedding + learned positions of the slice; image: the slice's pixels ‖ Fourier PE)."""
    from ..models.adapters import ImageInputAdapter, TextInputAdapter

    if isinstance(adapter, TextInputAdapter):
        return adapter.text_embedding(x[:, lo:hi]) * adapter.scale + adapter.pos_encoding[lo:hi].unsqueeze(0)
    if isinstance(adapter, ImageInputAdapter):
        adapter.check_shape(x)
        b = x.shape[0]
        pix = x.reshape(b, -1, adapter.num_image_channels)[:, lo:hi]
        pe = adapter.position_encoding[lo:hi].to(pix.dtype).unsqueeze(0).expand(b, -1, -1)
        return torch.cat([pix, pe], dim=-1)
    return adapter(x)[:, lo:hi]


class ContextParallelEncoder(nn.Module):
    """Runs a :class:`~perceiver_io_amd.models.PerceiverEncoder` with its M inputs sharded over
    ``group`` (default: the whole world).  Same parameters (it wraps, not copies, the encoder),
    same return value ``(x_latent, pad_mask)`` — the latent output is replicated on every rank."""

    def __init__(self, encoder, group=None, impl: Optional[str] = None):
        super().__init__()
        self.encoder = encoder
        self.group = group
        self.impl = impl  # "kernel" / "torch" / None (kernel on a GPU)

    def shard(self, m: int) -> Tuple[int, int]:
        return shard_range(m, _group_rank(self.group), _group_size(self.group))

    def forward(self, x, pad_mask=None):
        enc = self.encoder
        if self.training and any(isinstance(mod, nn.Dropout) and mod.p > 0 for mod in enc.modules()):
            raise ValueError("context parallelism requires dropout = 0 (replicated layers would diverge)")
        m = pad_mask.shape[1] if pad_mask is not None else _num_inputs(enc.input_adapter, x)
        lo, hi = self.shard(m)
        x_kv = shard_input(enc.input_adapter, x, lo, hi)
        pm = pad_mask[:, lo:hi] if pad_mask is not None else None
        b = x.shape[0]
        x_latent = enc.latent.unsqueeze(0).expand(b, -1, -1)
        for layer in enc.layers():
            cross, block = layer[0], layer[1]
            x_latent = cp_cross_attention_layer(cross, x_latent, x_kv, pm, self.group, self.impl)
            x_latent = block(x_latent)
        return x_latent, pad_mask


def _num_inputs(adapter, x) -> int:
    from ..models.adapters import ImageInputAdapter

    if isinstance(adapter, ImageInputAdapter):
        return int(math.prod(adapter.spatial_shape))
    return x.shape[1]


__all__ = ["ContextParallelEncoder", "cp_cross_attention", "cp_cross_attention_layer", "shard_input", "shard_range"]
