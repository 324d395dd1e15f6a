"""Rank-sharded sampler (Lightning ``replace_sampler_ddp: true``, ``scripts/trainer.yaml:61``;
SURVEY C-06): every rank sees a disjoint, equally sized shard; ``set_epoch`` reshuffles."""
from __future__ import annotations

import math
from typing import Iterator

import torch


class ShardedSampler(torch.utils.data.Sampler):
    def __init__(self, n: int, rank: int = 0, world_size: int = 1, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.n, self.rank, self.world = n, rank, world_size
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last:
            self.per_rank = n // world_size
        else:
            self.per_rank = math.ceil(n / world_size)
        self.total = self.per_rank * world_size

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if self.drop_last:
            idx = idx[: self.total]
        else:
            idx += idx[: self.total - len(idx)]
        return iter(idx[self.rank:self.total:self.world])

    def __len__(self) -> int:
        return self.per_rank
