"""Routing of latent self-attention blocks to the per-sample block kernels (csrc/sample_block.hip):
32 latents, 4 heads, C ∈ {64, 128} (the image configs and the LArTPC experiment), no dropout,
1..3 identical layers (4 would overflow the backward's slab segments / weight-gradient jobs with
the cross layers' pre / post folds); anything else keeps the per-layer kernels."""
import pytest

from perceiver_io_amd.models.blocks import self_attention_block
from perceiver_io_amd.ops import fused


def _specs(L, C, heads, p=0.0):
    return [fused.layer_spec_and_params(ly)[0] for ly in self_attention_block(L, C, heads, p)]


@pytest.mark.parametrize("L,C", [(3, 128), (3, 64), (1, 64), (2, 128)])
def test_qualifying_blocks(L, C):
    assert fused._sample_block_ok(_specs(L, C, 4), 32, 0.0, True)


@pytest.mark.parametrize("L,C,heads,n,p,cuda", [
    (3, 128, 4, 64, 0.0, True),    # not 32 latents
    (3, 256, 4, 32, 0.0, True),    # channel width
    (3, 64, 8, 32, 0.0, True),     # head count
    (5, 128, 4, 32, 0.0, True),    # too many layers
    (4, 128, 4, 32, 0.0, True),    # 4L + 4 slab segments > 16
    (3, 128, 4, 32, 0.1, True),    # dropout
    (3, 128, 4, 32, 0.0, False),   # CPU tensors
])
def test_non_qualifying_blocks(L, C, heads, n, p, cuda):
    assert not fused._sample_block_ok(_specs(L, C, heads), n, p, cuda)


@pytest.mark.parametrize("C", [64, 128])
def test_sample_block_emulation_matches_fp32_autograd(C):
    """The emulation of sb_fwd / sb_bwd / sb_wgrad (ops/emulation.py: the kernels' operands and
    bf16 rounding points, the oracle the GPU three-way tests run the fused executor on) against
    fp32 autograd of the same block: every output / gradient within 2 % (relative Frobenius)."""
    import math

    import torch

    from perceiver_io_amd.ops import emulation as E

    torch.manual_seed(C)
    B, L, N, H = 5, 2, 32, 4

    def rn(*s, sc=1.0):
        return (torch.randn(*s) * sc).requires_grad_()

    ps = [dict(g1=(1 + torch.randn(C) * 0.1).requires_grad_(), be1=rn(C, sc=0.1), wqkv=rn(3 * C, C, sc=0.08),
               bqkv=rn(3 * C, sc=0.05), wo=rn(C, C, sc=0.08), bo=rn(C, sc=0.05),
               g2=(1 + torch.randn(C) * 0.1).requires_grad_(), be2=rn(C, sc=0.1), w1=rn(C, C, sc=0.08),
               b1=rn(C, sc=0.05), w2=rn(C, C, sc=0.08), b2=rn(C, sc=0.05)) for _ in range(L)]
    x = torch.randn(B, N, C)
    F = torch.nn.functional

    def ref(x):
        d = C // H
        for p in ps:
            h = F.layer_norm(x, (C,), p["g1"], p["be1"], 1e-5)
            q, k, v = ((h @ p["wqkv"].t() + p["bqkv"]).split(C, -1))
            q, k, v = (t.reshape(B, N, H, d).transpose(1, 2) for t in (q, k, v))
            o = (torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), -1) @ v).transpose(1, 2).reshape(B, N, C)
            y = x + o @ p["wo"].t() + p["bo"]
            h2 = F.layer_norm(y, (C,), p["g2"], p["be2"], 1e-5)
            x = y + F.gelu(h2 @ p["w1"].t() + p["b1"]) @ p["w2"].t() + p["b2"]
        return x

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())

    xr = x.clone().requires_grad_()
    r = ref(xr)
    dz = torch.randn_like(r)
    r.backward(dz)
    kp = []
    for p in ps:
        b = {k: p[k].detach().to(torch.bfloat16) for k in ("wqkv", "wo", "w1", "w2")}
        kp += [p["g1"].detach(), p["be1"].detach(), b["wqkv"], p["bqkv"].detach(), b["wo"], p["bo"].detach(),
               p["g2"].detach(), p["be2"].detach(), b["w1"], p["b1"].detach(), b["w2"], p["b2"].detach()]
    sc = 1.0 / math.sqrt(C // H)
    sv = E.sb_fwd(x.view(-1, C), kp, sc, 1e-5)
    errs = {"z": rel(sv[12 * (L - 1) + 7].view(B, N, C), r.detach())}
    out = E.sb_bwd(dz.view(-1, C), x.view(-1, C), sv, kp, sc, 1e-5)
    errs["dx"] = rel(out[0].view(B, N, C), xr.grad)
    ln = out[1].sum(0).view(4 * L, C)  # the per-sample LayerNorm partial slab, reduced
    for i in range(L):
        dq, dy, du, dzz = out[2 + 4 * i:6 + 4 * i]
        s = sv[12 * i:12 * (i + 1)]
        for G, A, wn, bn in ((dq, s[0], "wqkv", "bqkv"), (dy, s[2], "wo", "bo"), (du, s[3], "w1", "b1"),
                             (dzz, s[5], "w2", "b2")):
            dW, db = torch.zeros_like(ps[i][wn]), torch.zeros_like(ps[i][bn])
            E.sb_wgrad([G, A, dW, db])
            errs[f"{wn}{i}"], errs[f"{bn}{i}"] = rel(dW, ps[i][wn].grad), rel(db, ps[i][bn].grad)
        for j, n in enumerate(("g1", "be1", "g2", "be2")):
            errs[f"{n}{i}"] = rel(ln[4 * i + j], ps[i][n].grad)
    bad = {k: v for k, v in errs.items() if not v < 2e-2}
    assert not bad, errs
