"""Data parallelism over RCCL/xGMI: process-group bootstrap, flat-buffer gradient reducer,
rank-sharded sampler, and a single-node launcher."""
from . import dist
from .reducer import FlatGradReducer
from .sampler import ShardedSampler

__all__ = ["dist", "FlatGradReducer", "ShardedSampler"]
