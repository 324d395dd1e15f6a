"""Small utilities: ``freeze`` (reference ``perceiver/utils.py:17-19``) and masked-token
prediction (``perceiver/utils.py:22-43``: top-k fill-ins at ``[MASK]`` positions)."""
from __future__ import annotations

import torch

from .tokenizer import MASK_TOKEN


def freeze(module: torch.nn.Module):
    for p in module.parameters():
        p.requires_grad = False


@torch.no_grad()
def predict_masked_samples(masked_samples, encode_fn, tokenizer, model, num_predictions: int = 5, device=None):
    """For each sample, ``num_predictions`` decoded strings: the i-th fills every ``[MASK]``
    with its i-th most likely token.  All variants are built as one ``(k, n, L)`` tensor and
    decoded with one ``decode_batch`` call."""
    ids, pad = (t.to(device) for t in encode_fn(masked_samples))
    mode = model.training
    model.eval()
    try:
        logits, _ = model(ids, pad, masking=False)
    finally:
        model.train(mode)
    at_mask = ids == tokenizer.token_to_id(MASK_TOKEN)                      # (n, L)
    top = logits[at_mask].float().topk(num_predictions, dim=-1).indices     # (masks, k)
    filled = ids.unsqueeze(0).repeat(num_predictions, 1, 1)                 # (k, n, L)
    filled[:, at_mask] = top.t().to(filled.dtype)
    n = ids.shape[0]
    texts = tokenizer.decode_batch(filled.reshape(num_predictions * n, -1).tolist(), skip_special_tokens=True)
    return [[texts[i * n + j] for i in range(num_predictions)] for j in range(n)]
