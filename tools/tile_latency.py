"""Per-kernel time vs. grid size at the headline self-attention layer shapes: how much of a
kernel is one tile's dependent-latency chain (1 workgroup) and how much is the full grid.

    python tools/tile_latency.py            (GPU)
"""
import math
import sys

import torch

sys.path.insert(0, ".")
from perceiver_io_amd.ops import ext  # noqa: E402
from tools.microbench import timeit  # noqa: E402


def main():
    global timeit
    bs = (1, 4, 16, 64)
    if len(sys.argv) > 1 and sys.argv[1] == "pmc":  # counter pass: each kernel 3× at B = 64, untimed
        bs = (64,)

        def timeit(fn, iters=3, warmup=0):  # noqa: F811
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            return 0.0
    K = ext.require()
    dev = "cuda"
    C, H, N = 64, 4, 256
    D = C // H
    bf = torch.bfloat16
    print(f"{'kernel':28s} " + " ".join(f"B={b:<6d}" for b in bs))
    rows = {}
    for B in bs:
        R = B * N
        x = torch.randn(R, C, device=dev)
        g1, b1 = torch.randn(C, device=dev), torch.randn(C, device=dev)
        wqkv = (torch.randn(3 * C, C, device=dev) / 8).to(bf)
        bqkv = torch.randn(3 * C, device=dev)
        rows.setdefault("ln_linear_fwd qkv", []).append(
            timeit(lambda: K.ln_linear_fwd(x, g1, b1, 1e-5, wqkv, bqkv, 0, None, True, True)))
        qkv, mean, rstd = K.ln_linear_fwd(x, g1, b1, 1e-5, wqkv, bqkv, 0, None, True, True)
        q3 = qkv.view(B, N, 3 * C)
        q, k, v = q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:]
        rows.setdefault("attn_fwd", []).append(timeit(lambda: K.attn_fwd(q, k, v, None, H, D, 1 / math.sqrt(D), 0.0, None, 1)))
        o, lse = K.attn_fwd(q, k, v, None, H, D, 1 / math.sqrt(D), 0.0, None, 1)
        ws = [(torch.randn(C, C, device=dev) / 8).to(bf) for _ in range(3)]
        bs = [torch.randn(C, device=dev) for _ in range(3)]
        g2, be2 = torch.randn(C, device=dev), torch.randn(C, device=dev)
        o2 = o.view(R, C)
        rows.setdefault("post_attn_fwd", []).append(
            timeit(lambda: K.post_attn_fwd(o2, x, ws[0], bs[0], g2, be2, 1e-5, ws[1], bs[1], ws[2], bs[2])))
        z, y, m2, r2, u = K.post_attn_fwd(o2, x, ws[0], bs[0], g2, be2, 1e-5, ws[1], bs[1], ws[2], bs[2])
        dz = torch.randn(R, C, device=dev)
        nt = (R + 63) // 64
        pa_sizes = [C * C, C, C, C, C * C, C, C * C, C]
        pa_offs = [sum(pa_sizes[:i]) for i in range(8)]
        pa_slab = torch.empty(nt, sum(pa_sizes), device=dev)
        pa_views = [pa_slab[:, o_:o_ + n] for o_, n in zip(pa_offs, pa_sizes)]
        rows.setdefault("post_attn_bwd (slab)", []).append(
            timeit(lambda: K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, pa_views, slab=True)))
        dy, do, delta = K.post_attn_bwd(dz, y, m2, r2, u, o2, ws[0], ws[1], ws[2], g2, be2, H, pa_views, slab=True)
        dqkv = torch.empty(B, N, 3 * C, device=dev)
        rows.setdefault("attn_bwd", []).append(
            timeit(lambda: K.attn_bwd(q, k, v, None, o, do.view(B, N, C), lse, delta.view(B, N, H), H, D,
                                      1 / math.sqrt(D), 0.0, None, dqkv[:, :, :C], dqkv[:, :, C:2 * C], dqkv[:, :, 2 * C:])))
        ll_sizes = [C, C, 3 * C * C, 3 * C]
        ll_offs = [sum(ll_sizes[:i]) for i in range(4)]
        ll_slab = torch.empty(nt, sum(ll_sizes), device=dev)
        ll_views = [ll_slab[:, o_:o_ + n] for o_, n in zip(ll_offs, ll_sizes)]
        g = dqkv.view(R, 3 * C)
        rows.setdefault("ln_linear_bwd (slab)", []).append(
            timeit(lambda: K.ln_linear_bwd(g, wqkv, x, mean, rstd, g1, b1, dy, True, *ll_views, slab=True)))
        e = torch.empty(1, device=dev)
        rows.setdefault("empty fill (launch floor)", []).append(timeit(lambda: e.zero_()))
    for k_, v_ in rows.items():
        print(f"{k_:28s} " + " ".join(f"{t:8.2f}" for t in v_))


if __name__ == "__main__":
    main()
