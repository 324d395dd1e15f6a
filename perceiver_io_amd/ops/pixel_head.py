"""Per-pixel classification head + class-weighted cross-entropy (SURVEY K-17) over the HIP
kernels of ``csrc/pixel_head.hip``.

``pixel_ce(h, linear, labels, weights)`` returns the loss of
``F.cross_entropy(linear(h), labels, weight=weights, ignore_index=-100)`` together with the
per-class accuracies of the LArTPC experiment (reference ``run.py:190-206``).  Logits never
reach memory: the forward pass reads each row of ``h`` once and writes per-block partial sums.
The backward pass reads it again and writes ``dH`` plus per-block ``dW | db`` partials, which are
summed in a fixed order (deterministic).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from . import ext


def _supported(h, w) -> bool:
    from . import use_hip

    return use_hip(h) and h.shape[-1] in (32, 64, 128) and 2 <= w.shape[0] <= 4


class _PixelCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, b, labels, wts):
        from .fused import kernels

        K = kernels(h)
        h2 = h.reshape(-1, h.shape[-1]).float().contiguous()
        lab = labels.reshape(-1).contiguous()
        stats, loss = K.pixel_ce_fwd(h2, w.contiguous(), b.contiguous(), lab, wts.float().contiguous())
        ctx.save_for_backward(h2, lab, wts, stats)
        ctx.w, ctx.b, ctx.hshape = w, b, h.shape
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        return loss, stats

    @staticmethod
    def backward(ctx, g, _gstats):
        from .fused import kernels

        if g is None:
            return None, None, None, None, None
        K = kernels(g)
        h2, lab, wts, stats = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        grads = []
        for p in (w, b):  # accumulated in place: flat-buffer gradient views stay bound
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad if p.requires_grad else torch.zeros_like(p))
        dh = torch.empty_like(h2)
        K.pixel_ce_bwd(h2, w.contiguous(), b.contiguous(), lab, wts.float().contiguous(), g.float().reshape(1).contiguous(),
                       stats, dh, grads[0], grads[1])
        return dh.view(ctx.hshape), None, None, None, None


def _metrics(stats: torch.Tensor, K: int) -> Dict[str, torch.Tensor]:
    ns = 4 + 2 * K
    out = {"acc": stats[ns]}
    for k in range(1, K):
        out[f"acc{k}"] = stats[ns + k]
    return out


def pixel_ce(h: torch.Tensor, linear: torch.nn.Linear, labels: torch.Tensor,
             weights: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """(weighted mean CE, {acc, acc1, …}) of ``linear(h)`` against ``labels`` (-100 ignored);
    ``acc`` over labels > 0, ``acc<k>`` over label k (device tensors, no host sync)."""
    K = linear.weight.shape[0]
    if _supported(h, linear.weight):
        loss, stats = _PixelCE.apply(h, linear.weight, linear.bias, labels, weights)
        return loss, _metrics(stats, K)
    logits = linear(h).reshape(-1, K).float()
    lab = labels.reshape(-1)
    loss = F.cross_entropy(logits, lab, weight=weights, ignore_index=-100)
    pred = logits.argmax(-1)
    out = {}
    for name, sel in [("acc", lab > 0)] + [(f"acc{k}", lab == k) for k in range(1, K)]:
        n = sel.sum()
        hit = ((pred == lab) & sel).sum()
        out[name] = torch.where(n > 0, hit.float() / n.clamp(min=1).float(), torch.zeros((), device=lab.device))
    return loss, out
