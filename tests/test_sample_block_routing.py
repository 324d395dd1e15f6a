"""Routing of latent self-attention blocks to the per-sample block kernels (csrc/sample_block.hip):
32 latents, 4 heads, C ∈ {64, 128} (the image configs and the LArTPC experiment), no dropout,
1..4 identical layers; anything else keeps the per-layer kernels."""
import pytest

from perceiver_io_amd.models.blocks import self_attention_block
from perceiver_io_amd.ops import fused


def _specs(L, C, heads, p=0.0):
    return [fused.layer_spec_and_params(ly)[0] for ly in self_attention_block(L, C, heads, p)]


@pytest.mark.parametrize("L,C", [(3, 128), (3, 64), (1, 64), (4, 128)])
def test_qualifying_blocks(L, C):
    assert fused._sample_block_ok(_specs(L, C, 4), 32, 0.0, True)


@pytest.mark.parametrize("L,C,heads,n,p,cuda", [
    (3, 128, 4, 64, 0.0, True),    # not 32 latents
    (3, 256, 4, 32, 0.0, True),    # channel width
    (3, 64, 8, 32, 0.0, True),     # head count
    (5, 128, 4, 32, 0.0, True),    # too many layers
    (3, 128, 4, 32, 0.1, True),    # dropout
    (3, 128, 4, 32, 0.0, False),   # CPU tensors
])
def test_non_qualifying_blocks(L, C, heads, n, p, cuda):
    assert not fused._sample_block_ok(_specs(L, C, heads), n, p, cuda)
