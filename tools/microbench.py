"""Kernel microbenchmarks at the headline (MLM-256) self-attention layer shapes.

    python tools/microbench.py            (GPU)

Times each HIP entry point with CUDA events over many launches (one stream, warm L2) and
prints µs per call; variants isolate costs (e.g. the weight-gradient atomics).
"""
import math
import sys

import torch

sys.path.insert(0, ".")
from perceiver_io_amd.ops import ext  # noqa: E402


def timeit(fn, iters=200, warmup=20):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    K = ext.require()
    dev = "cuda"
    B, N, C, H = 64, 256, 64, 4
    R = B * N
    D = C // H
    bf = torch.bfloat16
    x = torch.randn(R, C, device=dev)
    g1, b1 = torch.randn(C, device=dev), torch.randn(C, device=dev)
    wqkv = (torch.randn(3 * C, C, device=dev) / 8).to(bf)
    bqkv = torch.randn(3 * C, device=dev)
    res = {}
    res["ln_linear_fwd qkv"] = timeit(lambda: K.ln_linear_fwd(x, g1, b1, 1e-5, wqkv, bqkv, 0, None, True, True))
    qkv, mean, rstd = K.ln_linear_fwd(x, g1, b1, 1e-5, wqkv, bqkv, 0, None, True, True)
    q3 = qkv.view(B, N, 3 * C)
    q, k, v = q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:]
    res["attn_fwd self"] = timeit(lambda: K.attn_fwd(q, k, v, None, H, D, 1 / math.sqrt(D), 0.0, None, 1))
    o, lse = K.attn_fwd(q, k, v, None, H, D, 1 / math.sqrt(D), 0.0, None, 1)
    ws = [(torch.randn(C, C, device=dev) / 8).to(bf) for _ in range(3)]
    bs = [torch.randn(C, device=dev) for _ in range(3)]
    g2, be2 = torch.randn(C, device=dev), torch.randn(C, device=dev)
    o2 = o.view(R, C)
    res["post_attn_fwd"] = timeit(lambda: K.post_attn_fwd(o2, x, ws[0], bs[0], g2, be2, 1e-5, ws[1], bs[1], ws[2], bs[2]))
    z, y, m2, r2, u = K.post_attn_fwd(o2, x, ws[0], bs[0], g2, be2, 1e-5, ws[1], bs[1], ws[2], bs[2])
    dz = torch.randn(R, C, device=dev)
    grads = [torch.zeros((C, C) if i in (0, 4, 6) else (C,), device=dev) for i in range(8)]
    res["post_attn_bwd"] = timeit(lambda: K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, grads))
    dy, do, delta = K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, grads)
    dqkv = torch.empty(B, N, 3 * C, device=dev)
    res["attn_bwd self"] = timeit(lambda: K.attn_bwd(q, k, v, None, o, do.view(B, N, C), lse, delta.view(B, N, H), H, D,
                                                     1 / math.sqrt(D), 0.0, None, dqkv[:, :, :C], dqkv[:, :, C:2 * C],
                                                     dqkv[:, :, 2 * C:]))
    dg, db_ = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dW, dbias = torch.zeros(3 * C, C, device=dev), torch.zeros(3 * C, device=dev)
    g = dqkv.view(R, 3 * C)
    res["ln_linear_bwd qkv (+dW)"] = timeit(lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, dg, db_, dW, dbias))
    res["ln_linear_bwd qkv (no dW)"] = timeit(lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, dg, db_, None, None))
    res["ln_linear_bwd qkv (no dW, no LN)"] = timeit(
        lambda: K.ln_linear_bwd(g, wqkv, x, None, None, None, None, dy, True, None, None, None, None))
    res["wgrad standalone qkv"] = timeit(lambda: K.wgrad(g, x, 1, mean, rstd, g1, b1, 256, dW, dbias))
    # every target replicated (weights too)
    big = torch.zeros(8, 3 * C * C + 5 * C + 3 * C * C + 3 * C + 2 * C, device=dev)
    off = [0]

    def take(n):
        t = big[:, off[0]:off[0] + n]
        off[0] += n
        return t
    ga = [take(C * C), take(C), take(C), take(C), take(C * C), take(C), take(C * C), take(C)]
    res["post_attn_bwd (all targets replicated)"] = timeit(
        lambda: K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, ga))
    wq_r, bq_r, g_r, b_r = take(3 * C * C), take(3 * C), take(C), take(C)
    res["ln_linear_bwd qkv (all targets replicated)"] = timeit(
        lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, g_r, b_r, wq_r, bq_r))
    # per-tile slab sinks (plain stores) + the side-stream reduction, timed separately
    nt = (R + 63) // 64
    pa_sizes = [C * C, C, C, C, C * C, C, C * C, C]
    pa_offs = [sum(pa_sizes[:i]) for i in range(8)]
    pa_slab = torch.empty(nt, sum(pa_sizes), device=dev)
    pa_views = [pa_slab[:, o:o + n] for o, n in zip(pa_offs, pa_sizes)]
    res["post_attn_bwd (slab)"] = timeit(
        lambda: K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, pa_views, slab=True))
    res["slab_reduce post_attn"] = timeit(lambda: K.slab_reduce(pa_slab, [g.view(-1) for g in grads], pa_offs))
    ll_sizes = [C, C, 3 * C * C, 3 * C]
    ll_offs = [sum(ll_sizes[:i]) for i in range(4)]
    ll_slab = torch.empty(nt, sum(ll_sizes), device=dev)
    ll_views = [ll_slab[:, o:o + n] for o, n in zip(ll_offs, ll_sizes)]
    res["ln_linear_bwd qkv (slab)"] = timeit(
        lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, *ll_views, slab=True))
    res["slab_reduce qkv"] = timeit(lambda: K.slab_reduce(ll_slab, [dg, db_, dW.view(-1), dbias], ll_offs))
    pa_dsts = [t.view(-1) for t in grads]
    res["ln_linear_bwd qkv (slab) + post_attn job"] = timeit(
        lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, *ll_views, slab=True, job_slab=pa_slab,
                                job_dsts=pa_dsts, job_offs=pa_offs))
    ll_dsts = [dg, db_, dW.view(-1), dbias]
    res["post_attn_bwd (slab) + qkv job"] = timeit(
        lambda: K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, pa_views, slab=True,
                                job_slab=ll_slab, job_dsts=ll_dsts, job_offs=ll_offs))
    for k_, v_ in res.items():
        print(f"{k_:45s} {v_:8.2f} us")


if __name__ == "__main__":
    main()
