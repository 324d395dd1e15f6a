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
    n = len(masked_samples)
    xs, ms = encode_fn(masked_samples)
    xs, ms = xs.to(device), ms.to(device)
    was_training = model.training
    model.eval()
    try:
        logits, _ = model(xs, ms, masking=False)
    finally:
        model.train(was_training)
    pred_mask = xs == tokenizer.token_to_id(MASK_TOKEN)
    _, pred = torch.topk(logits[pred_mask].float(), k=num_predictions, dim=-1)
    out = xs.clone()
    dec = [[] for _ in range(n)]
    for i in range(num_predictions):
        out[pred_mask] = pred[:, i]
        for j in range(n):
            dec[j].append(tokenizer.decode(out[j].tolist(), skip_special_tokens=True))
    return dec
