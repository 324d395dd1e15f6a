"""Synthetic datasets with the shapes of the reference workloads (the GPU box has no network).

* ``SyntheticText``  — token-id sequences over a vocab with special ids 0..2 reserved
  (PAD/UNK/MASK), random lengths in [min_len, max_len], binary labels correlated with the
  tokens (so classifiers can learn); text is rendered as "w<id>" words so the WordPiece
  tokenizer path and masked-sample predictions work end-to-end.
* ``SyntheticImages`` — channels-last images (e.g. 28×28×1 MNIST, 224×224×3 ImageNet-shape)
  whose class is encoded as a spatial frequency pattern + noise.
* ``lartpc_event``   — a 512×512 sparse "wire-plane" image with a few line-shaped tracks and
  per-pixel 3-class labels (background / track / shower), standing in for the LArCV/ROOT
  input of the reference's ``run.py`` (larcv/ROOT are not available).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch


class SyntheticText(torch.utils.data.Dataset):
    def __init__(self, n: int, vocab_size: int, min_len: int, max_len: int, seed: int = 0, num_special: int = 3):
        self.n, self.vocab, self.min_len, self.max_len = n, vocab_size, min_len, max_len
        self.seed, self.num_special = seed, num_special

    def __len__(self):
        return self.n

    def ids(self, i: int) -> Tuple[int, List[int]]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        label = int(torch.randint(0, 2, (1,), generator=g))
        length = int(torch.randint(self.min_len, self.max_len + 1, (1,), generator=g))
        lo, hi = self.num_special, self.vocab
        mid = (lo + hi) // 2
        # label-dependent token distribution: class 1 prefers the upper half of the vocab
        base = torch.randint(lo, hi, (length,), generator=g)
        bias = torch.randint(mid if label else lo, hi if label else mid, (length,), generator=g)
        pick = torch.rand(length, generator=g) < 0.3
        return label, torch.where(pick, bias, base).tolist()

    def __getitem__(self, i):
        label, ids = self.ids(i)
        return label, " ".join(f"w{t}" for t in ids)


class SyntheticImages(torch.utils.data.Dataset):
    def __init__(self, n: int, image_shape: Tuple[int, int, int], num_classes: int, seed: int = 0,
                 channels_last: bool = True):
        self.n, self.shape, self.k, self.seed, self.cl = n, tuple(image_shape), num_classes, seed, channels_last

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        h, w, c = self.shape
        y = int(torch.randint(0, self.k, (1,), generator=g))
        yy, xx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
        f = 1.0 + (y % 7)
        ang = math.pi * y / max(1, self.k)
        pat = torch.sin(math.pi * f * (xx * math.cos(ang) + yy * math.sin(ang)))
        img = pat.unsqueeze(-1).expand(h, w, c) + 0.5 * torch.randn(h, w, c, generator=g)
        img = img.clamp(-1, 1)
        if not self.cl:
            img = img.permute(2, 0, 1).contiguous()
        return img.float(), y


def lartpc_event(seed: int, size: int = 512, n_tracks: int = 6, occupancy_min: float = 0.012):
    """(image (size, size) float32 ≥ 0, labels (size*size,) int64 in {0, 1, 2})."""
    g = torch.Generator().manual_seed(seed)
    img = torch.zeros(size, size)
    lab = torch.zeros(size, size, dtype=torch.long)
    while (img > 0).float().mean() < occupancy_min:
        for _ in range(n_tracks):
            cls = 1 if torch.rand(1, generator=g).item() < 0.6 else 2
            x0, y0 = torch.randint(0, size, (2,), generator=g).tolist()
            ang = torch.rand(1, generator=g).item() * math.pi
            length = int(torch.randint(40, 300, (1,), generator=g))
            width = 1 if cls == 1 else 4
            t = torch.arange(length).float()
            xs = (x0 + t * math.cos(ang)).long()
            ys = (y0 + t * math.sin(ang)).long()
            for dw in range(-width, width + 1):
                xi = (xs + dw).clamp(0, size - 1)
                yi = ys.clamp(0, size - 1)
                ok = (xs + dw >= 0) & (xs + dw < size) & (ys >= 0) & (ys < size)
                img[yi[ok], xi[ok]] = img[yi[ok], xi[ok]] + torch.rand(int(ok.sum()), generator=g) * 50 + 10
                lab[yi[ok], xi[ok]] = cls
    return img, lab.reshape(-1)


class SyntheticLArTPC(torch.utils.data.Dataset):
    def __init__(self, n: int, size: int = 512, seed: int = 0):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return lartpc_event(self.seed * 1_000_003 + i, self.size)
