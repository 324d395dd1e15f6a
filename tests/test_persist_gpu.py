"""The persistent self-attention block kernels (csrc/persist.hip): one launch for every layer of a
C = 64, H = 4 latent block (reference model.py:36-44, 185-187).

Per layer they run exactly the math of the per-layer chain kernels (chain.hip), so the block's
outputs must be BITWISE those of the per-layer launches; the emulation comparison bounds both.
The in-launch hand-offs between the tiles of one batch element are also exercised under uneven
load (a concurrent GEMM stream holding CUs) and with more tiles than one XCD's CUs.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
C, H = 64, 4


def _ext():
    from perceiver_io_amd.ops import ext

    return ext.require()


def _emu():
    from perceiver_io_amd.ops import emulation

    return emulation


def bf(x):
    return x.to(torch.bfloat16)


def rel_fro(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _block_params(L, last_q, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)

    def rn(*s, sc=1.0):
        return torch.randn(*s, device=DEV, generator=g) * sc

    def w(*s):
        return bf(rn(*s, sc=0.15))

    ps = dict(wo=[w(C, C) for _ in range(L)], bo=[rn(C, sc=0.1) for _ in range(L)],
              g2=[1 + rn(C, sc=0.1) for _ in range(L)], be2=[rn(C, sc=0.1) for _ in range(L)],
              w1=[w(C, C) for _ in range(L)], b1=[rn(C, sc=0.1) for _ in range(L)],
              w2=[w(C, C) for _ in range(L)], b2=[rn(C, sc=0.1) for _ in range(L)])
    nn = L - 1 + (1 if last_q else 0)
    ps.update(lnw=[1 + rn(C, sc=0.1) for _ in range(nn)], lnb=[rn(C, sc=0.1) for _ in range(nn)],
              wq=[w(3 * C if i < L - 1 else last_q, C) for i in range(nn)],
              bq=[rn(3 * C if i < L - 1 else last_q, sc=0.1) for i in range(nn)])
    return ps


def _per_layer(K, qkv, x, N, ps, seed, p):
    """the block as one sa_layer_fwd launch per layer (chain.hip), flattened like sa_block_fwd"""
    out = []
    L = len(ps["wo"])
    for i in range(L):
        nx = i < len(ps["wq"])
        extra = dict(lnw=ps["lnw"][i], lnb=ps["lnb"][i], wq=ps["wq"][i], bq=ps["bq"][i]) if nx else {}
        r = K.sa_layer_fwd(qkv, x, N, 0.25, ps["wo"][i], ps["bo"][i], ps["g2"][i], ps["be2"][i], 1e-5, ps["w1"][i],
                           ps["b1"][i], ps["w2"][i], ps["b2"][i], seed=seed, site=i, p=p, **extra)
        out += list(r)
        x = r[2]
        qkv = r[7] if nx else None
    return out


def _block(K, qkv, x, N, ps, seed, p):
    return K.sa_block_fwd(qkv, x, N, 0.25, 1e-5, ps["wo"], ps["bo"], ps["g2"], ps["be2"], ps["w1"], ps["b1"], ps["w2"],
                          ps["b2"], ps["lnw"], ps["lnb"], ps["wq"], ps["bq"], seed=seed, p=p)


@pytest.mark.parametrize("B,N,L,last_q,p", [(64, 256, 6, 64, 0.0), (5, 256, 3, 0, 0.1), (7, 128, 2, 128, 0.0),
                                           (9, 64, 6, 0, 0.0), (3, 192, 1, 64, 0.0), (300, 64, 2, 0, 0.1)])
def test_sa_block_fwd_bitwise_per_layer(B, N, L, last_q, p):
    """One persistent launch == L per-layer launches, bit for bit, and within 2 % (relative
    Frobenius) of the fp32 emulation on every output; no hand-off wait timed out.  last_q: rows
    of the last layer's projection (0: none, 64 / 128: a following cross-attention layer's query /
    K-V projection)."""
    torch.manual_seed(3)
    K = _ext()
    R = B * N
    qkv = bf(torch.randn(R, 3 * C, device=DEV))
    x = torch.randn(R, C, device=DEV)
    ps = _block_params(L, last_q, seed=B + N + L)
    seed = torch.tensor([424242], dtype=torch.int64, device=DEV) if p > 0 else None
    K.persist_errors(True)
    a = _block(K, qkv, x, N, ps, seed, p)
    assert a, "sa_block_fwd did not take the operands"
    b = _per_layer(K, qkv, x, N, ps, seed, p)
    torch.cuda.synchronize()
    assert K.persist_errors(True) == 0
    assert len(a) == len(b)
    diff = [i for i, (u, v) in enumerate(zip(a, b)) if not torch.equal(u, v)]
    assert not diff, f"outputs {diff} differ from the per-layer kernels"
    if B <= 9:
        e = _block(_emu(), qkv, x, N, ps, seed, p)
        errs = [rel_fro(u, v) for u, v in zip(a, e)]
        assert max(errs) < 2e-2, errs


def test_sa_block_fwd_under_concurrent_load():
    """The in-launch hand-offs with another stream's GEMMs occupying CUs (tiles start late and
    unevenly; workgroups need not be co-resident): still bitwise the per-layer result, no timeout."""
    torch.manual_seed(4)
    K = _ext()
    B, N, L = 128, 256, 6  # 512 tiles: two rounds of workgroups
    R = B * N
    qkv = bf(torch.randn(R, 3 * C, device=DEV))
    x = torch.randn(R, C, device=DEV)
    ps = _block_params(L, 0, seed=7)
    ref = _per_layer(K, qkv, x, N, ps, None, 0.0)
    side = torch.cuda.Stream()
    a_ = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    K.persist_errors(True)
    for it in range(4):
        with torch.cuda.stream(side):
            for _ in range(3):
                a_ = (a_ @ a_).clamp_(-1, 1)
        out = _block(K, qkv, x, N, ps, None, 0.0)
        torch.cuda.synchronize()
        assert all(torch.equal(u, v) for u, v in zip(out, ref)), f"iteration {it}"
    assert K.persist_errors(True) == 0


def test_sa_block_fwd_graph_replay():
    """Captured in a hipGraph and replayed with other work in the graph that reuses freed memory:
    the sync words are reset by each launch's last workgroup, so every replay recomputes the
    eager result (the outputs are poisoned before each replay)."""
    torch.manual_seed(5)
    K = _ext()
    B, N, L = 16, 256, 3
    R = B * N
    qkv = bf(torch.randn(R, 3 * C, device=DEV))
    x = torch.randn(R, C, device=DEV)
    ps = _block_params(L, 64, seed=9)
    ref = _block(K, qkv, x, N, ps, None, 0.0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _block(K, qkv, x, N, ps, None, 0.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _block(K, qkv, x, N, ps, None, 0.0)
        junk = [torch.empty(1000 + i, device=DEV).fill_(1.0) * 2 for i in range(20)]  # noqa: F841
    K.persist_errors(True)
    for _ in range(3):
        for t in out:
            t.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(u, v) for u, v in zip(out, ref))
        assert K.persist_errors(True) == 0
