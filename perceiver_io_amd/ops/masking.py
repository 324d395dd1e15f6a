"""BERT-style text masking (reference ``perceiver/model.py:265-293``).

Both backends draw the same three uniforms per token with ``torch.rand`` (graph-capture
safe) and the random replacement ids with ``torch.randint`` over the full batch, then
select without any host synchronisation; the HIP path does the select in one kernel.
Unlike the reference, the input ids are never modified in place (defect D4).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import ext


def text_masking(x: torch.Tensor, pad_mask: Optional[torch.Tensor], vocab_size: int, unk_token_id: int,
                 mask_token_id: int, num_special_tokens: int, mask_p: float = 0.15,
                 generator: Optional[torch.Generator] = None):
    u = torch.rand((3,) + tuple(x.shape), device=x.device, generator=generator)
    rid = torch.randint(num_special_tokens, vocab_size, x.shape, device=x.device, generator=generator)
    from . import use_hip

    if use_hip(x):
        pm = pad_mask.to(torch.bool).contiguous() if pad_mask is not None else None
        xm, labels = ext.text_mask(x.contiguous(), pm, u.contiguous(), rid.contiguous(), unk_token_id,
                                   mask_token_id, mask_p)
        return xm, labels
    special = x == unk_token_id
    if pad_mask is not None:
        special = special | pad_mask
    sel = ~special & (u[0] < mask_p)
    msk = sel & (u[1] < 0.9)
    rnd = msk & (u[2] < 1.0 / 9.0)
    xm = torch.where(rnd, rid, torch.where(msk, torch.full_like(x, mask_token_id), x))
    labels = torch.where(sel, x, torch.full_like(x, -100))
    return xm, labels
