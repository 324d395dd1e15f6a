"""perceiver_io_amd — a Perceiver IO training framework built for AMD Instinct MI355X (gfx950).

Layers: ``models`` (parameter layout + eager oracle), ``ops`` (HIP/CDNA4 kernels behind
autograd Functions, fused layer executor, fused optimizer), ``parallel`` (RCCL data
parallelism), ``train`` (trainer, Lightning-layout checkpoints, HIP-graph step capture),
``cli`` (LightningCLI-compatible flags), ``data`` (IMDB / MNIST / synthetic).
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401
from .models import *  # noqa: F401,F403
