"""Sparse batches for the LArTPC experiment (``models/lartpc.py``).

A LArTPC wire-plane image is ~1–3 % non-zero.  ``sparse_collate`` turns dense events
``(image (H, W), labels (H·W,))`` into fixed-capacity sparse tensors, on the CPU inside the
DataLoader workers:

* ``values`` (B, K, 1) float32 — the non-zero pixel values, ``index`` (B, K) int64 — their flat
  positions, ``kmask`` (B, K) bool — True on capacity padding (masked keys);
* ``qidx`` (B, Q) int64 — the pixels with a non-zero class weight (the only ones the weighted
  loss sees), ``qlab`` (B, Q) int64 — their labels, -100 on padding.

K and Q are the batch maxima rounded up to a multiple of ``bucket``.  That gives a handful of
distinct shapes, so the step engine keeps one captured hipGraph per shape.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ..models.lartpc import CLASS_WEIGHTS


def _round_up(n: int, m: int) -> int:
    return max(m, -(-n // m) * m)


def sparse_collate(events: List[Tuple[torch.Tensor, torch.Tensor]], bucket: int = 2048,
                   weights: Sequence[float] = CLASS_WEIGHTS):
    w = torch.tensor(list(weights))
    keys, queries = [], []
    for img, lab in events:
        flat = img.reshape(-1)
        nz = torch.nonzero(flat != 0).squeeze(1)
        keys.append((flat[nz], nz))
        q = torch.nonzero(w[lab.reshape(-1)] > 0).squeeze(1)
        queries.append((q, lab.reshape(-1)[q]))
    b = len(events)
    K = _round_up(max(len(k[1]) for k in keys), bucket)
    Q = _round_up(max(len(q[0]) for q in queries), bucket)
    values = torch.zeros(b, K, 1)
    index = torch.zeros(b, K, dtype=torch.long)
    kmask = torch.ones(b, K, dtype=torch.bool)
    # unused query slots point at distinct pixels (their zero gradients then never pile onto one
    # row of the output-query table in the gather's backward)
    npix = events[0][1].numel()
    qidx = (torch.arange(Q) % npix).repeat(b, 1)
    qlab = torch.full((b, Q), -100, dtype=torch.long)
    for i, ((v, nz), (q, ql)) in enumerate(zip(keys, queries)):
        n, m = len(nz), len(q)
        values[i, :n, 0] = v
        index[i, :n] = nz
        kmask[i, :n] = False
        qidx[i, :m] = q
        qlab[i, :m] = ql
    return values, index, kmask, qidx, qlab


class SparseCollator:
    """Picklable ``collate_fn`` for DataLoader workers."""

    def __init__(self, bucket: int = 2048, weights: Sequence[float] = CLASS_WEIGHTS):
        self.bucket, self.weights = bucket, tuple(weights)

    def __call__(self, events):
        return sparse_collate(events, self.bucket, self.weights)
