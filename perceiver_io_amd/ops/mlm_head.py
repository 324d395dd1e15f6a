"""Masked-LM head: vocab projection + cross-entropy over the selected positions only.

Reference: ``TextOutputAdapter`` (``perceiver/adapter.py:166-173``) + ``CrossEntropyLoss``
over ``(B, V, L)`` (``perceiver/lightning.py:223-226``).  Since decoder queries never
interact, evaluating the head only where ``label != -100`` gives the identical mean loss
and gradients at ~15 % of the cost.

HIP path: rows are compacted on device into a fixed-capacity index list (no host sync,
graph-capturable; capacity = expected count + 8σ + 64, overflow probability < 1e-15 and
reported through :func:`last_overflow`), then one fused kernel pair computes logits tile
by tile in registers (``csrc/mlm_head.hip``) — the logits are never written to memory.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import ext

_overflow = None


def last_overflow():
    """Device bool of the most recent HIP call: True if selected rows exceeded capacity."""
    return _overflow


def capacity(n_positions: int, p: float = 0.15) -> int:
    mu = n_positions * p
    cap = int(math.ceil(mu + 8.0 * math.sqrt(max(mu * (1 - p), 1.0)) + 64))
    return max(1, min(n_positions, cap))


class _MaskedCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias, idx, labels_c, count):
        c = h.shape[-1]
        hs = h.reshape(-1, c).index_select(0, idx).to(torch.bfloat16).contiguous()
        wb = weight.to(torch.bfloat16).contiguous()
        loss_rows, lse = ext.ce_fwd(hs, labels_c, wb, bias.contiguous())
        denom = count.clamp(min=1).to(torch.float32)
        ctx.save_for_backward(hs, wb, bias, lse, idx, labels_c, denom)
        ctx.hshape = h.shape
        ctx.weight, ctx.bias_p = weight, bias
        return loss_rows.sum() / denom

    @staticmethod
    def backward(ctx, g):
        hs, wb, bias, lse, idx, labels_c, denom = ctx.saved_tensors
        weight = ctx.weight
        gscale = (g.to(torch.float32) / denom).reshape(1).contiguous()
        d_rows = torch.zeros(hs.shape, device=hs.device, dtype=torch.float32)
        # vocab-head parameter gradients are accumulated in place into .grad (flat buffer views)
        for p in (weight, ctx.bias_p):
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        ext.ce_bwd(hs, labels_c, wb, bias.contiguous(), lse, gscale, d_rows, weight.grad, ctx.bias_p.grad, True)
        shp = ctx.hshape
        dh = torch.zeros((shp[0] * shp[1], shp[2]), device=hs.device, dtype=torch.float32)
        dh.index_add_(0, idx, d_rows)
        return dh.view(shp), None, None, None, None, None


def compact_rows(labels: torch.Tensor, cap: int):
    """Fixed-capacity compaction of ``labels != -100`` → (idx[cap], labels[cap], count)."""
    global _overflow
    flat = labels.reshape(-1)
    n = flat.numel()
    sel = flat != -100
    count = sel.sum()
    pos = torch.cumsum(sel.to(torch.int32), 0) - 1
    target = torch.where(sel & (pos < cap), pos, torch.full_like(pos, cap)).to(torch.int64)
    buf = torch.zeros(cap + 1, dtype=torch.int64, device=labels.device)
    buf.scatter_(0, target, torch.arange(n, device=labels.device, dtype=torch.int64))
    idx = buf[:cap]
    valid = torch.arange(cap, device=labels.device) < count
    labels_c = torch.where(valid, flat.index_select(0, idx), torch.full_like(idx, -100)).contiguous()
    _overflow = count > cap
    return idx, labels_c, count


def masked_lm_loss(h: torch.Tensor, labels: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor):
    """Mean CE over positions with ``label != -100``; ``h`` is ``(B, L, C)``."""
    from . import use_hip

    if use_hip(h) and h.shape[-1] in (32, 64, 128):
        cap = capacity(labels.numel())
        idx, labels_c, count = compact_rows(labels, cap)
        return _MaskedCE.apply(h, weight, bias, idx, labels_c, count)
    sel = labels.reshape(-1) != -100
    hs = h.reshape(-1, h.shape[-1])[sel]
    logits = F.linear(hs, weight, bias)
    if hs.shape[0] == 0:
        return logits.sum() * 0.0
    return F.cross_entropy(logits.float(), labels.reshape(-1)[sel])
