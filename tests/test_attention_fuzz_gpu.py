"""Shape fuzzing of the flash attention kernels (d ∈ {16, 32, 128}, N ∈ {1 … 512},
ragged key-padding masks, fully masked rows) against the fp32 emulation, with hypothesis.

Each example draws a head width, query / key counts, batch sizes (broadcast queries included),
a split-KV count and a mask pattern (none, ragged suffix padding as the IMDB collator makes it,
random, a fully padded batch row); forward O / LSE and backward dQ / dK / dV must match the
emulation within 1 % relative Frobenius error (2 % for dQ / dK / dV of long rows, which sum
bf16 products over up to 512 keys), and fully masked rows give exactly zero (defect D10).
"""
import math

import pytest
import torch

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda"
NS = (1, 2, 3, 31, 32, 33, 64, 100, 255, 256, 257, 512)


def _rel(a, b, floor=0.0):
    """relative Frobenius error; ``floor``: per-element magnitude below which a reference is
    treated as zero (dQ of a single key is 0 in exact arithmetic, ~1e-7 after bf16 rounding)"""
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), floor * b.numel() ** 0.5, 1e-30)).item()


@st.composite
def attn_case(draw):
    D = draw(st.sampled_from([16, 32, 128]))
    H = draw(st.sampled_from([1, 2, 4]))
    Nq = draw(st.sampled_from(NS))
    Nk = draw(st.sampled_from(NS))
    B = draw(st.integers(1, 3))
    Bq = draw(st.sampled_from([1, B]))
    ns = draw(st.sampled_from([1, 2, 4]))
    mask = draw(st.sampled_from(["none", "ragged", "random", "dead_row"]))
    seed = draw(st.integers(0, 2**31 - 1))
    return D, H, Nq, Nk, B, Bq, ns, mask, seed


@settings(max_examples=40, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(attn_case())
def test_attention_shapes_fuzz(case):
    from perceiver_io_amd.ops import emulation, ext

    K = ext.require()
    D, H, Nq, Nk, B, Bq, ns, mask, seed = case
    g = torch.Generator(device=DEV).manual_seed(seed)
    E = H * D
    q = torch.randn(Bq, Nq, E, device=DEV, generator=g).to(torch.bfloat16)
    kv = torch.randn(B, Nk, 2 * E, device=DEV, generator=g).to(torch.bfloat16)
    k, v = kv[:, :, :E], kv[:, :, E:]
    km = None
    if mask == "ragged":  # suffix padding, one length per batch row
        lens = torch.randint(1, Nk + 1, (B,), generator=torch.Generator().manual_seed(seed))
        km = (torch.arange(Nk)[None, :] >= lens[:, None]).to(DEV)
    elif mask == "random":
        km = torch.rand(B, Nk, device=DEV, generator=g) < 0.3
    elif mask == "dead_row":
        km = torch.rand(B, Nk, device=DEV, generator=g) < 0.3
        km[0] = True
    scale = 1.0 / math.sqrt(D)
    ns = min(ns, max(1, (Nk + 127) // 128))
    o1, l1 = K.attn_fwd(q, k, v, km, H, D, scale, 0.0, None, ns)
    o2, l2 = emulation.attn_fwd(q, k, v, km, H, D, scale, 0.0, None, ns)
    assert _rel(o1, o2) < 1e-2, ("O", case)
    fin = torch.isfinite(l2)
    assert torch.equal(torch.isfinite(l1), fin), ("LSE pattern", case)
    if fin.any():
        assert _rel(l1[fin], l2[fin]) < 1e-3, ("LSE", case)
    if mask == "dead_row":  # every key of batch row 0 padded: defined as zero output
        assert o1[0].float().abs().max().item() == 0.0, ("dead row", case)
    do = torch.randn(max(B, Bq), Nq, E, device=DEV, generator=g).to(torch.bfloat16)
    ga = K.attn_bwd(q, k, v, km, o1, do, l1, None, H, D, scale, 0.0, None, None, None, None)
    gb = emulation.attn_bwd(q, k, v, km, o1, do, l1, None, H, D, scale, 0.0, None, None, None, None)
    tol = 2e-2 if max(Nq, Nk) > 256 else 1e-2
    for a, b, n in zip(ga, gb, ("dq", "dk", "dv")):
        err = _rel(a, b, floor=1e-3)
        assert err < tol, (n, err, case)


@pytest.mark.parametrize("D,H,Nk,B,Bq", [(128, 1, 32, 3, 1), (128, 2, 64, 2, 2), (128, 1, 1, 2, 2)])
def test_decode_attention_shapes(D, H, Nk, B, Bq):
    """The few-key one-query shapes of the classifier decoders (csrc/attention.hip
    attn_decode_bwd_kernel for head width 128): the fuzz test's checks at fixed cases, plus the
    backward accumulating onto existing dK / dV (a weight-shared layer's later application)."""
    from perceiver_io_amd.ops import emulation, ext

    test_attention_shapes_fuzz.hypothesis.inner_test((D, H, 1, Nk, B, Bq, 1, "none", 7 * D + Nk))
    if Nk == 1:  # one key: dK is zero up to rounding, nothing to compare an accumulation against
        return
    K = ext.require()
    g = torch.Generator(device=DEV).manual_seed(D + Nk)
    E = H * D
    q = torch.randn(Bq, 1, E, device=DEV, generator=g).to(torch.bfloat16)
    kv = torch.randn(B, Nk, 2 * E, device=DEV, generator=g).to(torch.bfloat16)
    k, v = kv[:, :, :E], kv[:, :, E:]
    scale = 1.0 / math.sqrt(D)
    o, lse = K.attn_fwd(q, k, v, None, H, D, scale, 0.0, None, 1)
    do = torch.randn(B, 1, E, device=DEV, generator=g).to(torch.bfloat16)
    dkv = torch.randn(B, Nk, 2 * E, device=DEV, generator=g)
    base = dkv.clone()
    K.attn_bwd(q, k, v, None, o, do, lse, None, H, D, scale, 0.0, None, None, dkv[:, :, :E], dkv[:, :, E:], True)
    ref = emulation.attn_bwd(q, k, v, None, o, do, lse, None, H, D, scale, 0.0, None, None, None, None)
    assert _rel(dkv[:, :, :E] - base[:, :, :E], ref[1], floor=1e-3) < 1e-2
    assert _rel(dkv[:, :, E:] - base[:, :, E:], ref[2], floor=1e-3) < 1e-2
