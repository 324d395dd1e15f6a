"""Synthetic datasets with the shapes of the reference workloads (the GPU box has no network).

* ``SyntheticText``  — token-id sequences over a vocab with special ids 0..2 reserved
  (PAD/UNK/MASK), random lengths in [min_len, max_len], binary labels; text is rendered as
  "w<id>" words so the WordPiece tokenizer path and masked-sample predictions work end-to-end.
  ``structure="topic"`` (default) mixes three sources per position, the way real text is
  layered: a Zipf-distributed global vocabulary, a per-document topic vocabulary (16 topics;
  label = topic parity) and a sparse Markov successor of the previous token.  An MLM first
  learns the Zipf marginal, then the document topic from context, then the local transitions —
  a loss curve with the structure convergence checks need.  ``"markov"`` uses only the two
  label chains; ``"unigram"`` keeps i.i.d. tokens with a label-dependent bias.
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


MARKOV_PROBS = (0.55, 0.25, 0.12, 0.08)  # successor probabilities (plus MARKOV_NOISE uniform jumps)
MARKOV_NOISE = 0.1


def markov_tables(vocab_size: int, num_special: int = 3, seed: int = 1234) -> torch.Tensor:
    """(2, V, 4) successor ids of the two label chains (ids ≥ num_special)."""
    g = torch.Generator().manual_seed(seed + vocab_size)
    return torch.randint(num_special, vocab_size, (2, vocab_size, len(MARKOV_PROBS)), generator=g)


TOPICS = 16
TOPIC_SIZE = 64
TOPIC_MIX = (0.45, 0.3, 0.25)  # P(global Zipf), P(topic vocabulary), P(Markov successor)


def topic_tables(vocab_size: int, num_special: int = 3, seed: int = 4321):
    """(zipf_cdf (V-ns,), zipf_ids (V-ns,), topic_ids (TOPICS, TOPIC_SIZE), successors (V, 4))."""
    g = torch.Generator().manual_seed(seed + vocab_size)
    n = vocab_size - num_special
    w = 1.0 / torch.arange(1, n + 1, dtype=torch.float64)
    cdf = (w / w.sum()).cumsum(0).float()
    ids = torch.randperm(n, generator=g) + num_special
    topics = torch.randint(num_special, vocab_size, (TOPICS, TOPIC_SIZE), generator=g)
    succ = torch.randint(num_special, vocab_size, (vocab_size, len(MARKOV_PROBS)), generator=g)
    return cdf, ids, topics, succ


def topic_batch(tables, topic: torch.Tensor, L: int, g: torch.Generator):
    """(B, L) token ids for documents of the given topics (label = topic % 2)."""
    cdf, ids, topics, succ = tables
    B = topic.shape[0]
    glob = ids[torch.searchsorted(cdf, torch.rand(B, L, generator=g)).clamp(max=ids.numel() - 1)]
    tpk = topics[topic[:, None], torch.randint(0, TOPIC_SIZE, (B, L), generator=g)]
    src = torch.rand(B, L, generator=g)
    cum = torch.tensor(MARKOV_PROBS).cumsum(0)[:-1]
    choice = (torch.rand(B, L, generator=g)[..., None] > cum).sum(-1)
    base = torch.where(src < TOPIC_MIX[0], glob, tpk)
    markov = src >= TOPIC_MIX[0] + TOPIC_MIX[1]
    out = base.clone()
    for t in range(1, L):
        out[:, t] = torch.where(markov[:, t], succ[out[:, t - 1], choice[:, t]], base[:, t])
    return out


def markov_batch(tables: torch.Tensor, labels: torch.Tensor, L: int, g: torch.Generator, num_special: int = 3):
    """(B, L) token ids: a walk on chain ``labels[b]`` per row.  The random draws are made for
    the whole (B, L) block at once; the walk itself is a cheap gather per position."""
    B = labels.shape[0]
    V = tables.shape[1]
    cum = torch.tensor(MARKOV_PROBS).cumsum(0)[:-1]
    u = torch.rand(B, L, generator=g)
    choice = (u[..., None] > cum).sum(-1)                       # successor slot per step
    jump = torch.rand(B, L, generator=g) < MARKOV_NOISE
    rnd = torch.randint(num_special, V, (B, L), generator=g)
    out = torch.empty(B, L, dtype=torch.long)
    state = rnd[:, 0]
    tab = tables[labels]                                        # (B, V, 4)
    rows = torch.arange(B)
    for t in range(L):
        out[:, t] = state
        state = torch.where(jump[:, t], rnd[:, t], tab[rows, state, choice[:, t]])
    return out


class SyntheticText(torch.utils.data.Dataset):
    def __init__(self, n: int, vocab_size: int, min_len: int, max_len: int, seed: int = 0, num_special: int = 3,
                 structure: str = "topic"):
        if structure not in ("topic", "markov", "unigram"):
            raise ValueError(f"structure must be 'topic', 'markov' or 'unigram', got {structure!r}")
        self.n, self.vocab, self.min_len, self.max_len = n, vocab_size, min_len, max_len
        self.seed, self.num_special, self.structure = seed, num_special, structure
        self.tables = (markov_tables(vocab_size, num_special) if structure == "markov" else
                       topic_tables(vocab_size, num_special) if structure == "topic" else None)

    def __len__(self):
        return self.n

    def ids(self, i: int) -> Tuple[int, List[int]]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        label = int(torch.randint(0, 2, (1,), generator=g))
        length = int(torch.randint(self.min_len, self.max_len + 1, (1,), generator=g))
        if self.structure == "topic":
            topic = int(torch.randint(0, TOPICS // 2, (1,), generator=g)) * 2 + label
            return label, topic_batch(self.tables, torch.tensor([topic]), length, g)[0].tolist()
        if self.tables is not None:
            return label, markov_batch(self.tables, torch.tensor([label]), length, g, self.num_special)[0].tolist()
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
                 channels_last: bool = True, noise: float = 0.5, random_phase: bool = False):
        """``noise`` (pixel noise std) and ``random_phase`` (a random shift of the class
        pattern per image) set the difficulty; the defaults give an easily separable set."""
        self.n, self.shape, self.k, self.seed, self.cl = n, tuple(image_shape), num_classes, seed, channels_last
        self.noise, self.random_phase = noise, random_phase

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        h, w, c = self.shape
        y = int(torch.randint(0, self.k, (1,), generator=g))
        yy, xx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
        f = 1.0 + (y % 7)
        ang = math.pi * y / max(1, self.k)
        phase = float(torch.rand(1, generator=g)) * 2 * math.pi if self.random_phase else 0.0
        pat = torch.sin(math.pi * f * (xx * math.cos(ang) + yy * math.sin(ang)) + phase)
        img = pat.unsqueeze(-1).expand(h, w, c) + self.noise * torch.randn(h, w, c, generator=g)
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
