"""Masked-LM head: vocab projection + cross-entropy over the selected positions only.

Reference: ``TextOutputAdapter`` (``perceiver/adapter.py:166-173``) + ``CrossEntropyLoss``
over ``(B, V, L)`` (``perceiver/lightning.py:223-226``).  Since decoder queries never
interact, evaluating the head only where ``label != -100`` gives the identical mean loss
and gradients at ~15 % of the cost.

HIP path: rows are compacted on device into a fixed-capacity index list (no host sync,
graph-capturable; capacity = expected count + 8σ + 64 at the masking rate ``p`` of the model's
``TextMasking``, overflow probability < 1e-15), then one fused kernel pair computes logits tile
by tile in registers (``csrc/mlm_head.hip``) — the logits are never written to memory.

Overflow is never silent: every call ORs its device overflow bit into a persistent per-device
flag (an in-place op, so replayed hipGraphs update it too); the trainer reads it at log steps
(:func:`check_overflow`) and raises.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import ext

_overflow = None
_flags = {}


def last_overflow():
    """Device bool of the most recent call: True if selected rows exceeded capacity."""
    return _overflow


def overflow_flag(device) -> torch.Tensor:
    """Persistent device bool: set once any call on ``device`` overflowed its capacity."""
    device = torch.device(device)
    f = _flags.get(device)
    if f is None:
        f = _flags[device] = torch.zeros((), dtype=torch.bool, device=device)
    return f


def _record(ovf: torch.Tensor):
    global _overflow
    _overflow = ovf
    overflow_flag(ovf.device).logical_or_(ovf.reshape(()))


def check_overflow(reset: bool = False) -> bool:
    """Host check (one sync) of every device's overflow flag; raises if any is set."""
    hit = [d for d, f in _flags.items() if bool(f.item())]
    if reset:
        for f in _flags.values():
            f.zero_()
    if hit:
        raise RuntimeError(f"masked-LM selected positions exceeded the fixed row capacity on {hit}: "
                           "labels fell out of the loss.  The capacity follows TextMasking.mask_p — "
                           "check that the masking rate passed to the loss matches the model's")
    return False


def capacity(n_positions: int, p: float = 0.15) -> int:
    p = min(max(float(p), 1e-6), 1.0)
    mu = n_positions * p
    cap = int(math.ceil(mu + 8.0 * math.sqrt(max(mu * (1 - p), 1.0)) + 64))
    return max(1, min(n_positions, cap))


class _MaskedCE(torch.autograd.Function):
    """Mean CE over rows ``idx`` of ``h`` (``idx=None``: every row, ``h`` already compacted).

    The forward reads the fp32 rows of ``h`` through ``idx`` and leaves their compact bf16 copy
    for the backward (no separate gather / cast kernels), finalises
    the mean ``Σ rows / max(count, 1)`` in the combine kernel and form the row-loss gradient
    ``g / max(count, 1)`` on the device: no framework kernels around the head."""

    @staticmethod
    def forward(ctx, h, weight, bias, idx, labels_c, count):
        c = h.shape[-1]
        h2 = h.reshape(-1, c)
        if h2.dtype != torch.float32 or not h2.is_contiguous():
            h2 = h2.float().contiguous()
        count_labels = count is None  # the combine kernel counts the rows with a label itself
        if count_labels:
            cnt = torch.empty(1, device=h2.device, dtype=torch.float32)
        else:
            cnt = count.reshape(1)
            if cnt.dtype != torch.float32:
                cnt = cnt.to(torch.float32)
        from .fused import weight_cache

        wb = weight_cache.get(weight)  # bf16 shadow written by the fused optimizer
        # the backward's dH accumulator (atomic partials) is cleared by the forward kernel
        dh = torch.empty((h2.shape[0], c), device=h2.device, dtype=torch.float32)
        outs = ext.ce_fwd(h2, idx, labels_c, wb, bias.contiguous(), cnt, dh, count_labels)
        loss, lse, hs = outs[:3]
        # C = 64: the two-pass head also returns the per-split Σ_v p·W partials of every row and
        # the splits' (max, sum): the backward merges them into the hidden-state gradient rows, so
        # it makes only the dW / db pass over the vocabulary
        ctx.u = (outs[3], outs[4]) if len(outs) > 4 else None
        ctx.dh = dh
        ctx.save_for_backward(hs, wb, bias, lse, idx if idx is not None else torch.empty(0, dtype=torch.int64),
                              labels_c, cnt)
        ctx.hshape = h.shape
        ctx.hrows = h2.shape[0]
        ctx.weight, ctx.bias_p = weight, bias
        return loss

    @staticmethod
    def backward(ctx, g):
        hs, wb, bias, lse, idx, labels_c, cnt = ctx.saved_tensors
        weight = ctx.weight
        gout = g.reshape(1)
        if gout.dtype != torch.float32:
            gout = gout.to(torch.float32)
        # vocab-head parameter gradients are accumulated in place into .grad (flat buffer views);
        # the hidden-state gradient rows land straight at their source positions (rowmap)
        for p in (weight, ctx.bias_p):
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        shp = ctx.hshape
        dh, ctx.dh = ctx.dh, None
        from . import fused

        ix = idx if idx.numel() else None
        u, ctx.u = ctx.u, None
        slab = ext.ce_bwd(hs, labels_c, wb, bias.contiguous(), lse, gout.contiguous(), cnt, dh, weight.grad,
                          ctx.bias_p.grad, True, ix, slab=fused.WGRAD_SLAB, u=u[0] if u else None,
                          u_ml=u[1] if u else None)
        if slab is not None:  # dW / db row-split partials: reduced by the next backward kernel
            fused.defer_slab(ext, slab, [weight.grad.view(-1), ctx.bias_p.grad.view(-1)], [0, weight.numel()])
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
    _record(count > cap)
    return idx, labels_c, count


def masked_lm_loss(h: torch.Tensor, labels: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                   p: float = 0.15):
    """Mean CE over positions with ``label != -100``; ``h`` is ``(B, L, C)``; ``p`` the
    masking rate (sizes the row capacity)."""
    from . import use_hip

    if use_hip(h) and h.shape[-1] in (32, 64, 128):
        cap = capacity(labels.numel(), p)
        idx, labels_c, count = compact_rows(labels, cap)
        return _MaskedCE.apply(h, weight, bias, idx, labels_c, count)
    sel = labels.reshape(-1) != -100
    hs = h.reshape(-1, h.shape[-1])[sel]
    logits = F.linear(hs, weight, bias)
    if hs.shape[0] == 0:
        return logits.sum() * 0.0
    return F.cross_entropy(logits.float(), labels.reshape(-1)[sel])


# ------------------------------------------------------------------------------------------
# training-time decode of the selected positions only
# ------------------------------------------------------------------------------------------
def row_capacity(length: int, p: float = 0.15) -> int:
    """Per-sequence slots for selected positions: expected + 8σ + 16, a multiple of 32, ≤ L
    (L = 512, p = 0.15: 160 slots for ~77 selected; overflow probability < 1e-15 per sequence)."""
    p = min(max(float(p), 1e-6), 1.0)
    mu = length * p
    cap = int(math.ceil(mu + 8.0 * math.sqrt(max(mu * (1 - p), 1.0)) + 16))
    cap = (cap + 31) // 32 * 32
    return max(1, min(length, cap))


def compact_per_row(labels: torch.Tensor, cap: int):
    """Sync-free per-sequence compaction of ``labels != -100``: positions ``(B, cap)``, their
    labels (-100 in unused slots) and the total count."""
    global _overflow
    B, L = labels.shape
    sel = labels != -100
    pos = torch.cumsum(sel.to(torch.int32), 1) - 1
    target = torch.where(sel & (pos < cap), pos, torch.full_like(pos, cap)).to(torch.int64)
    # unused slots point at distinct positions (slot mod L): their zero gradients then do not
    # pile onto one output-query row in the gather's backward
    buf = (torch.arange(cap + 1, device=labels.device, dtype=torch.int64) % L).repeat(B, 1)
    buf.scatter_(1, target, torch.arange(L, device=labels.device, dtype=torch.int64).expand(B, L).contiguous())
    idx = buf[:, :cap].contiguous()
    cnt = sel.sum(1, keepdim=True)
    valid = torch.arange(cap, device=labels.device) < cnt
    labels_c = torch.where(valid, labels.gather(1, idx), torch.full_like(idx, -100))
    _record((cnt > cap).any())
    return idx, labels_c, sel.sum()


def compact_lm_loss(h: torch.Tensor, labels_c: torch.Tensor, count: torch.Tensor, weight: torch.Tensor,
                    bias: torch.Tensor, positions: int, p: float = 0.15):
    """Mean CE over the rows of a per-sequence-compacted ``(B, cap, C)`` batch whose label is
    not -100.  The HIP path compacts those rows once more over the whole batch (capacity for
    ``positions`` tokens at the masking rate), so the vocab GEMMs see only real rows."""
    from . import use_hip

    if use_hip(h) and h.shape[-1] in (32, 64, 128):
        idx, lab, cnt = compact_rows(labels_c, capacity(positions, p))
        return _MaskedCE.apply(h, weight, bias, idx, lab, cnt)
    lab = labels_c.reshape(-1)
    logits = F.linear(h.reshape(-1, h.shape[-1]), weight, bias)
    return F.cross_entropy(logits.float(), lab, ignore_index=-100, reduction="sum") / count.clamp(min=1)


def _index_add_grad(p: torch.nn.Parameter, idx: torch.Tensor, g: torch.Tensor):
    """``p.grad[idx] += g`` straight into the (flat-buffer) gradient: one kernel, no autograd
    zeros + index_add + AccumulateGrad."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    from . import deterministic, use_hip

    if deterministic():
        p.grad.index_put_((idx,), g.reshape(-1, p.grad.shape[1]).to(p.grad.dtype), accumulate=True)
    elif use_hip(g) and p.grad.dim() == 2 and p.grad.is_contiguous() and p.grad.shape[1] % 4 == 0:
        from .fused import kernels

        src = g.reshape(-1, p.grad.shape[1]).to(p.grad.dtype).contiguous()
        kernels(g).index_add_rows(p.grad, idx.contiguous(), src)
    else:
        p.grad.index_add_(0, idx, g.reshape(-1, p.grad.shape[1]).to(p.grad.dtype))


class _GatherQueries(torch.autograd.Function):
    """``param.index_select(0, idx)`` whose backward index-adds straight into ``param.grad``."""

    @staticmethod
    def forward(ctx, param, idx):
        from . import use_hip

        ctx.save_for_backward(idx)
        ctx.param = param
        if (use_hip(param) and param.dim() == 2 and param.dtype == torch.float32 and param.is_contiguous()
                and param.shape[1] % 4 == 0 and idx.dtype == torch.int64):
            from .fused import kernels

            return kernels(param).gather_rows(param.detach(), idx.contiguous())
        return param.index_select(0, idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            _index_add_grad(ctx.param, idx, g)
        return None, None


class _SelectQueries(torch.autograd.Function):
    """HIP path: one kernel selects the masked positions (per-sequence slots + global
    compaction) and gathers their output queries ``q = param[idx]`` (B, cap, C); the backward
    index-adds dq into ``param.grad``.  → q, idx (B, cap), gidx, glab, total, overflow."""

    @staticmethod
    def forward(ctx, param, labels, cap, gcap, sticky):
        idx, _, gidx, glab, total, ovf, q = ext.require().mlm_select(labels.contiguous(), cap, gcap, sticky,
                                                                     param.detach().contiguous())
        ctx.save_for_backward(idx)
        ctx.param = param
        ctx.mark_non_differentiable(idx, gidx, glab, total, ovf)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the index outputs
        return q, idx, gidx, glab, total, ovf

    @staticmethod
    def backward(ctx, g, *_):
        (idx,) = ctx.saved_tensors
        if g is not None and ctx.needs_input_grad[0]:
            _index_add_grad(ctx.param, idx.reshape(-1), g)
        return None, None, None, None, None


def masked_decode_loss(decoder, x_latent: torch.Tensor, labels: torch.Tensor, p: float = 0.15):
    """MLM loss decoding only the selected positions.

    Decoder queries never interact (reference ``perceiver/model.py:236``: one cross-attention
    from the K output queries to the latents), so decoding the ~15 % selected positions of each
    sequence — gathered into ``row_capacity(L, p)`` slots — gives the same loss and gradients as
    decoding all ``L`` at a third of the decoder cost.  The output-query
    gradient flows back through the gather (index_select → index_add).  ``p`` is the masking
    rate (``TextMasking.mask_p``): it sizes both capacities.
    """
    from ..parallel.reducer import bucket_ready_point
    from . import use_hip

    x_latent = bucket_ready_point(x_latent, decoder, "decoder")  # before any decoder op (DDP)
    B, L = labels.shape
    decoder.check_latent(x_latent)
    lin = decoder.output_adapter.linear
    cap = row_capacity(L, p)
    if use_hip(x_latent) and lin.weight.shape[1] in (32, 64, 128):
        # the kernel ORs the overflow into the persistent per-device flag itself
        q, idx, gidx, glab, total, ovf = _SelectQueries.apply(decoder.output, labels, cap, capacity(B * L, p),
                                                              overflow_flag(labels.device).view(1))
        global _overflow
        _overflow = ovf
        h = decoder.cross_attention(q, x_latent)
        return _MaskedCE.apply(h, lin.weight, lin.bias, gidx, glab, total)
    idx, labels_c, count = compact_per_row(labels, cap)
    q = _GatherQueries.apply(decoder.output, idx.reshape(-1)).view(B, cap, -1)
    h = decoder.cross_attention(q, x_latent)
    return compact_lm_loss(h, labels_c, count, lin.weight, lin.bias, B * L, p)


def classification_loss(decoder, x_latent: torch.Tensor, labels: torch.Tensor):
    """``cross_entropy(decoder(x_latent), labels)`` for a one-query classification decoder
    (``ClassificationOutputAdapter``, reference ``perceiver/adapter.py:138-143`` +
    ``lightning.py:61-66``).  HIP path: the class projection and the softmax cross-entropy run
    in the fused CE kernels over the decoder's (B, C) output rows — no logits tensor and no
    framework GEMM / reduction kernels; mean over the labels that are not ``-100``."""
    from . import use_hip

    h = decoder.hidden(x_latent)
    ad = decoder.output_adapter
    lin = getattr(ad, "linear", None)
    if (lin is not None and use_hip(h) and h.dim() == 3 and h.shape[1] == 1 and h.shape[-1] in (32, 64, 128)
            and labels.dim() == 1 and labels.shape[0] == h.shape[0]):
        lab = labels if labels.dtype == torch.int64 and labels.is_contiguous() else labels.to(torch.int64).contiguous()
        return _MaskedCE.apply(h, lin.weight, lin.bias, None, lab, None)  # count: rows with a label, in-kernel
    return F.cross_entropy(ad(h).float(), labels)

