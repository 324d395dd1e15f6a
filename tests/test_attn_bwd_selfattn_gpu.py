"""The latent self-attention backward with bf16 dQ / dK / dV (the operands of the chain-layout
layer-boundary kernel; reference ``perceiver/model.py:59-74`` inside the self-attention block of
``model.py:36-44``) at the C = 64, H = 4 latent shapes against the fp32 emulation
(``ops/emulation.py:attn_bwd``): the full-LDS 8-wave workgroup, and the two-query-tile variant
that carries the previous kernel's slab reduction in appended workgroups (whose result must equal
the standalone reduction's).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def _case(B, N, H=4, D=16, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    E = H * D
    qkv = torch.randn(B, N, 3 * E, device=DEV, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, :E], qkv[:, :, E:2 * E], qkv[:, :, 2 * E:]
    do = torch.randn(B, N, E, device=DEV, generator=g).to(torch.bfloat16)
    return q, k, v, do


def _fwd(K, q, k, v, do, H, D, scale):
    B, N = q.shape[0], q.shape[1]
    o, lse = K.attn_fwd(q, k, v, None, H, D, scale, 0.0, None, 1)
    delta = (do.float().view(B, N, H, D) * o.float().view(B, N, H, D)).sum(-1).contiguous()
    return o, lse, delta


@pytest.mark.parametrize("carry", [False, True])
@pytest.mark.parametrize("B,N", [(64, 256), (3, 256), (4, 128), (2, 192)])
def test_selfattn_bwd_bf16(B, N, carry):
    from perceiver_io_amd.ops import emulation, ext

    K = ext.require()
    H, D = 4, 16
    E = H * D
    scale = 1.0 / math.sqrt(D)
    q, k, v, do = _case(B, N, H, D, seed=B * 1000 + N)
    o, lse, delta = _fwd(K, q, k, v, do, H, D, scale)
    ref = emulation.attn_bwd(q, k, v, None, o, do, lse, delta, H, D, scale, 0.0, None, None, None, None)
    dqkv = torch.full((B, N, 3 * E), float("nan"), device=DEV).to(torch.bfloat16)
    job = {}
    if carry:  # a slab reduction of 64 rows × 1000 columns into two targets
        g = torch.Generator(device=DEV).manual_seed(5)
        slab = torch.randn(64, 1024, device=DEV, generator=g)
        t0, t1 = torch.zeros(600, device=DEV), torch.zeros(400, device=DEV)
        job = dict(job_slab=slab, job_dsts=[t0, t1], job_offs=[0, 600])
    K.attn_bwd(q, k, v, None, o, do, lse, delta, H, D, scale, 0.0, None, dqkv[:, :, :E], dqkv[:, :, E:2 * E],
               dqkv[:, :, 2 * E:], **job)
    torch.cuda.synchronize()
    assert torch.isfinite(dqkv.float()).all()
    for got, want, name in zip((dqkv[:, :, :E], dqkv[:, :, E:2 * E], dqkv[:, :, 2 * E:]), ref, ("dq", "dk", "dv")):
        err = _rel(got.float(), want.float())
        assert err < 1.5e-2, f"{name}: rel err {err:.3e}"
    if carry:
        s = slab.sum(0)
        assert _rel(t0, s[:600]) < 1e-5 and _rel(t1, s[600:1000]) < 1e-5


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("B,Nq,Nk", [(128, 64, 64), (3, 33, 64), (4, 64, 48)])
def test_few_key_selfattn_bwd_two_wave(B, Nq, Nk, p):
    """Head width 16 over ≤ 64 keys (the text classifiers' / MLM-64's latent self-attention,
    reference README.md:91-107): the two-wave workgroup (64 keys) instead of eight waves of which
    six would sweep padded keys; no key mask, attention-probability dropout on and off."""
    from perceiver_io_amd.ops import emulation, ext

    K = ext.require()
    H, D = 4, 16
    E = H * D
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=DEV).manual_seed(B + Nq + Nk)
    q = torch.randn(B, Nq, E, device=DEV, generator=g).to(torch.bfloat16)
    kv = torch.randn(B, Nk, 2 * E, device=DEV, generator=g).to(torch.bfloat16)
    k, v = kv[:, :, :E], kv[:, :, E:]
    do = torch.randn(B, Nq, E, device=DEV, generator=g).to(torch.bfloat16)
    sd = torch.tensor([31337], dtype=torch.int64, device=DEV) if p > 0 else None
    o, lse = K.attn_fwd(q, k, v, None, H, D, scale, p, sd, 1, site=2)
    ga = K.attn_bwd(q, k, v, None, o, do, lse, None, H, D, scale, p, sd, None, None, None, site=2)
    gb = emulation.attn_bwd(q, k, v, None, o, do, lse, None, H, D, scale, p, sd, None, None, None, site=2)
    torch.cuda.synchronize()
    for a, b, n in zip(ga, gb, ("dq", "dk", "dv")):
        err = _rel(a.float(), b.float())
        assert err < 2e-2, f"{n}: rel err {err:.3e}"


@pytest.mark.parametrize("B,p,gbf,nq", [(3, 0.0, False, 192), (8, 0.1, True, 192), (5, 0.1, False, 192),
                                        (4, 0.1, False, 64)])
def test_boundary_kernel_with_fused_attention_backward(B, p, gbf, nq):
    """64 latents per sample (the README MLM / text classifiers, reference README.md:33-44,
    91-107): the layer-boundary backward kernel with layer l's attention backward fused in
    (csrc/chain.hip phase D, ``att_*`` operands) against the same boundary kernel followed by the
    standalone attention backward: the chain outputs and slab partials unchanged, dQKV within
    bf16 rounding (with attention-probability dropout: the forward's hash stream).  nq = 64: the
    boundary with the next cross-attention layer's query projection above the block."""
    from perceiver_io_amd.ops import ext
    from perceiver_io_amd.ops.fused import PA_SIZES, _GradSlab

    K = ext.require()
    torch.manual_seed(31 + B)
    C, H, D, N = 64, 4, 16, 64
    R = B * N
    scale = 1.0 / math.sqrt(D)
    eps = 1e-5

    def w(*s, sc=0.15):
        return (torch.randn(*s, device=DEV) * sc).to(torch.bfloat16)

    x = torch.randn(R, C, device=DEV)
    mean1, rstd1 = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + eps)
    y = torch.randn(R, C, device=DEV)
    m2, r2 = y.mean(1), torch.rsqrt(y.var(1, unbiased=False) + eps)
    g = torch.randn(R, nq, device=DEV)
    if gbf:
        g = g.to(torch.bfloat16)
    dres = torch.randn(R, C, device=DEV)
    u = w(R, C, sc=1.0)
    wq, wo, w1, w2 = w(nq, C), w(C, C), w(C, C), w(C, C)
    lnw, lnb = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    g2, be2 = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    seed = torch.tensor([987654321], dtype=torch.int64, device=DEV) if p > 0 else None
    # layer l's attention operands (its forward's O feeds the post-attention backward)
    qkv = w(R, 3 * C, sc=1.0)
    q3 = qkv.view(B, N, 3 * C)
    o, lse = K.attn_fwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], None, H, D, scale, p, seed, 1, site=3)
    o = o.view(R, C)
    res = {}
    for fused in (False, True):
        sl = _GradSlab(R, [C, C, nq * C, nq] + PA_SIZES(C), x)
        sl.t.fill_(float("nan"))
        tg = sl.targets()
        att = {}
        if fused:
            out = torch.full((R, 3 * C), float("nan"), device=DEV).to(torch.bfloat16)
            att = dict(att_qkv=qkv, att_lse=lse, att_out=out, att_scale=scale)
        dy, dO, delta = K.ln_linear_post_attn_bwd(g, wq, x, mean1, rstd1, lnw, lnb, dres, tg[:4], y, m2, r2, u, o, wo,
                                                  w1, w2, g2, be2, H, tg[4:], seed=seed, site=3, p=p, **att)
        if not fused:
            d3 = torch.empty(B, N, 3 * C, device=DEV)
            K.attn_bwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], None, o.view(B, N, C), dO.view(B, N, C), lse,
                       delta.view(B, N, H), H, D, scale, p, seed, d3[:, :, :C], d3[:, :, C:2 * C], d3[:, :, 2 * C:],
                       site=3)
            out = d3.view(R, 3 * C)
        torch.cuda.synchronize()
        assert torch.isfinite(sl.t).all() and torch.isfinite(out.float()).all()
        res[fused] = (dy, sl.t.clone(), out.float())
    (dy0, s0, o0), (dy1, s1, o1) = res[False], res[True]
    assert torch.equal(dy0, dy1)
    assert torch.equal(s0, s1)
    for name, sl_ in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
        err = _rel(o1[:, sl_], o0[:, sl_])
        assert err < 1e-2, f"{name}: rel err {err:.3e}"
