"""Multi-head attention core: eager oracle and the HIP flash kernel.

Semantics (``nn.MultiheadAttention`` as used at reference ``perceiver/model.py:59-74``,
SURVEY App. A.2): ``softmax((q·d^-½)·kᵀ + mask)`` with ``-inf`` at padded keys,
dropout on the probabilities (training), ``P·v``, heads merged.  A query row whose keys
are *all* padded yields 0 here (the reference yields NaN; defect D10 defined).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from . import ext


def _split(x, h):
    b, n, e = x.shape
    return x.reshape(b, n, h, e // h).transpose(1, 2)


def mha_core(q, k, v, num_heads: int, key_padding_mask=None, attn_mask=None, dropout_p: float = 0.0):
    """Eager attention core on projected ``q (B, Nq, E)``, ``k, v (B, Nk, E)`` → ``(B, Nq, E)``."""
    if q.is_cuda and attn_mask is None and _hip_ok(q, num_heads):
        from . import use_hip

        if use_hip(q):
            return flash_attention(q, k, v, num_heads, key_padding_mask, dropout_p)
    b, nq, e = q.shape
    d = e // num_heads
    qh, kh, vh = _split(q, num_heads), _split(k, num_heads), _split(v, num_heads)
    s = torch.matmul(qh * (1.0 / math.sqrt(d)), kh.transpose(-1, -2))
    if attn_mask is not None:
        am = attn_mask
        if am.dtype == torch.bool:
            am = torch.zeros_like(am, dtype=s.dtype).masked_fill(am, float("-inf"))
        s = s + am
    dead = None
    if key_padding_mask is not None:
        kpm = key_padding_mask.view(b, 1, 1, -1)
        s = s.masked_fill(kpm, float("-inf"))
        dead = kpm.all(dim=-1, keepdim=True)
    p = torch.softmax(s, dim=-1)
    if dead is not None:
        p = p.masked_fill(dead, 0.0)
    if dropout_p > 0.0:
        p = F.dropout(p, p=dropout_p, training=True)
    o = torch.matmul(p, vh)
    return o.transpose(1, 2).reshape(b, nq, e)


def _hip_ok(q, num_heads) -> bool:
    e = q.shape[-1]
    return e % num_heads == 0 and (e // num_heads) in (16, 32, 64, 128)


def pick_splits(batch: int, heads: int, nq: int, nk: int, dropout: bool = False) -> int:
    """Split-KV factor so that few-query / many-key launches still fill 256 CUs."""
    waves = max(1, min(4, (nq + 31) // 32))
    blocks = ((nq + 32 * waves - 1) // (32 * waves)) * heads * batch
    tiles = (nk + 63) // 64
    if blocks >= 512:
        # ≥ 2 workgroups per CU already: a split only adds the combine launch — except for
        # 1-2-wave workgroups (≤ 64 queries, at most one wave per SIMD) doing the dropout hash
        # per score: the text classifier's cross-attention at batch 128 ran 28.6 → 18.5 µs
        # (+ a 4.8 µs combine); without dropout (15 µs) the combine eats the gain (r6)
        return 2 if dropout and blocks * waves < 2048 and tiles >= 8 else 1
    if not dropout and blocks * waves >= 512 and tiles < 16:
        # ≥ 2 waves per CU over a short key range: the 64-latent MLM cross-attention (256 two-wave
        # workgroups, 512 keys) runs 9.3 µs unsplit against 12.0 µs split in two with its
        # combine (tools/fwd_split_sweep.py, r6)
        return 1
    want = max(1, 1024 // max(blocks, 1))
    return int(max(1, min(want, tiles // 4 if tiles >= 8 else 1)))


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, kmask, heads, dropout_p, seed):
        d = q.shape[-1] // heads
        scale = 1.0 / math.sqrt(d)
        b = k.shape[0]
        nsplit = pick_splits(b, heads, q.shape[1], k.shape[1], dropout_p > 0)
        qb, kb, vb = (t.to(torch.bfloat16) for t in (q, k, v))
        o, lse = ext.attn_fwd(qb, kb, vb, kmask, heads, d, scale, dropout_p, seed, nsplit)
        ctx.save_for_backward(qb, kb, vb, kmask if kmask is not None else torch.empty(0), o, lse)
        ctx.cfg = (heads, d, scale, dropout_p, seed, kmask is not None, q.dtype, q.shape[0])
        return o.to(q.dtype) if q.dtype != torch.bfloat16 else o

    @staticmethod
    def backward(ctx, do):
        qb, kb, vb, km, o, lse = ctx.saved_tensors
        heads, d, scale, p, seed, has_mask, dt, bq = ctx.cfg
        dq, dk, dv = ext.attn_bwd(qb, kb, vb, km if has_mask else None, o, do.to(torch.bfloat16).contiguous(), lse,
                                  None, heads, d, scale, p, seed, None, None, None)
        if bq == 1 and dq.shape[0] > 1:
            dq = dq.sum(0, keepdim=True)
        return dq.to(dt), dk.to(dt), dv.to(dt), None, None, None, None


def flash_attention(q, k, v, num_heads: int, key_padding_mask: Optional[torch.Tensor] = None,
                    dropout_p: float = 0.0, seed: Optional[torch.Tensor] = None):
    """HIP flash attention on ``(B|1, Nq, E)`` queries and ``(B, Nk, E)`` keys/values.

    ``seed``: 1-element int64 device tensor for the dropout masks; drawn here on the device
    (graph-safe: a fresh draw on every replay of a captured step) when not given."""
    ext.require()
    if seed is None and dropout_p > 0:
        seed = torch.randint(-(2**62), 2**62, (1,), device=q.device, dtype=torch.int64)
    km = None
    if key_padding_mask is not None:
        km = key_padding_mask.to(torch.bool).contiguous()
    return _FlashAttention.apply(q, k, v, km, num_heads, float(dropout_p), seed)
