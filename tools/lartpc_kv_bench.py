"""Timing variants of the LArTPC encoder's K/V-projection LayerNorm + linear backward (sparse
execution: R = batch x capacity gathered pixel rows, Kin = 1 pixel + 130 Fourier-PE channels read
from the PE table at flat pixel indices, N = 2C = 128) and of its forward, to locate the cost of
`ln_linear_bwd_kernel<float, float, 5, false>` in the LArTPC step.

    python tools/lartpc_kv_bench.py [--rows 32768]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, iters=100, warmup=10):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    args = ap.parse_args()
    from perceiver_io_amd.ops import ext

    K = ext.require()
    dev = "cuda"
    R, Kin, N, M = args.rows, 131, 128, 512 * 512
    g = torch.Generator(device=dev).manual_seed(0)
    pe = torch.randn(M, 136, device=dev, generator=g)
    idx = torch.randint(0, M, (R,), device=dev, generator=g).sort().values
    x = torch.randn(R, 1, device=dev, generator=g)
    w = (torch.randn(N, 136, device=dev, generator=g) / 12).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g)
    lnw, lnb = torch.randn(Kin, device=dev, generator=g), torch.randn(Kin, device=dev, generator=g)
    res = {}
    res["ln_linear_fwd (bf16 out, stats)"] = timeit(
        lambda: K.ln_linear_fwd(x, lnw, lnb, 1e-5, w, bias, 0, None, True, True, pe, Kin, idx))
    y, mean, rstd = K.ln_linear_fwd(x, lnw, lnb, 1e-5, w, bias, 0, None, True, True, pe, Kin, idx)
    G = torch.randn(R, N, device=dev, generator=g)
    nt = (R + 63) // 64
    sizes = [Kin, Kin, N * Kin, N]
    offs = [sum(sizes[:i]) for i in range(4)]
    slab = torch.empty(nt, sum(sizes), device=dev)
    views = [slab[:, o:o + n] for o, n in zip(offs, sizes)]
    dg, db_ = torch.zeros(Kin, device=dev), torch.zeros(Kin, device=dev)
    dW, dbias = torch.zeros(N, Kin, device=dev), torch.zeros(N, device=dev)

    def bwd(**kw):
        return lambda: K.ln_linear_bwd(G, w, x, mean, rstd, lnw, lnb, None, False, **kw, pe=pe, kin=Kin, pe_index=idx)

    res["ln_linear_bwd slab (dLN + dW)"] = timeit(bwd(dlnw=views[0], dlnb=views[1], dW=views[2], db=views[3], slab=True))
    res["ln_linear_bwd atomic (dLN + dW)"] = timeit(bwd(dlnw=dg, dlnb=db_, dW=dW, db=dbias))
    res["ln_linear_bwd dLN only"] = timeit(bwd(dlnw=dg, dlnb=db_, dW=None, db=None))
    res["slab_reduce"] = timeit(lambda: K.slab_reduce(slab, [dg, db_, dW.view(-1), dbias], offs))
    Gb = G.to(torch.bfloat16)
    res["ln_linear_bwd slab, bf16 G"] = timeit(
        lambda: K.ln_linear_bwd(Gb, w, x, mean, rstd, lnw, lnb, None, False, dlnw=views[0], dlnb=views[1],
                                dW=views[2], db=views[3], slab=True, pe=pe, kin=Kin, pe_index=idx))
    for k_, v_ in res.items():
        print(f"{k_:40s} {v_:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
