"""Data parallelism over RCCL/xGMI: process-group bootstrap, flat-buffer gradient reducer,
rank-sharded sampler, a single-node launcher, and context parallelism for the encoder
(inputs sharded over ranks, partial softmax states combined by all-reduce)."""
from . import dist
from .context import ContextParallelEncoder
from .reducer import FlatGradReducer
from .sampler import ShardedSampler

__all__ = ["dist", "ContextParallelEncoder", "FlatGradReducer", "ShardedSampler"]
