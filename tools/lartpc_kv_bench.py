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


def timeit(fn, iters=100, warmup=10, name=None):
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
    class _R(dict):
        def __setitem__(self, k, v):
            print(f"{k:40s} {v:8.2f} us", flush=True)
            super().__setitem__(k, v)
    res = _R()
    res["ln_linear_fwd (bf16 out, stats)"] = timeit(
        lambda: K.ln_linear_fwd(x, lnw, lnb, 1e-5, w, bias, 0, None, True, True, pe, Kin, idx))
    y, mean, rstd = K.ln_linear_fwd(x, lnw, lnb, 1e-5, w, bias, 0, None, True, True, pe, Kin, idx)
    G = torch.randn(R, N, device=dev, generator=g)
    nt = (R + 63) // 64
    sizes = [Kin, Kin, N * Kin, N]
    pads = [(n + 3) // 4 * 4 for n in sizes]
    offs = [sum(pads[:i]) for i in range(4)]
    slab = torch.empty(nt, sum(pads), device=dev)
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

    # slab targets without the weight gradient (no same-address atomics)
    res["ln_linear_bwd slab (dLN only)"] = timeit(bwd(dlnw=views[0], dlnb=views[1], dW=None, db=None, slab=True))
    # row-count scaling of the step's variant
    for rr in (8192, 16384, 65536):
        Gr = torch.randn(rr, N, device=dev, generator=g)
        ir = torch.randint(0, M, (rr,), device=dev, generator=g).sort().values
        xr = torch.randn(rr, 1, device=dev, generator=g)
        _, mr, sr = K.ln_linear_fwd(xr, lnw, lnb, 1e-5, w, bias, 0, None, True, True, pe, Kin, ir)
        ntr = (rr + 63) // 64
        slr = torch.empty(ntr, sum(pads), device=dev)
        vr = [slr[:, o:o + n] for o, n in zip(offs, sizes)]
        res[f"ln_linear_bwd slab R={rr}"] = timeit(
            lambda: K.ln_linear_bwd(Gr, w, xr, mr, sr, lnw, lnb, None, False, vr[0], vr[1], vr[2], vr[3], pe=pe,
                                    kin=Kin, slab=True, pe_index=ir))
    # dense input rows, no PE split: Kin = 128 (every operand vectorised) and Kin = 131
    for kin2 in (128, 131):
        X2 = torch.randn(R, kin2, device=dev, generator=g)
        w2 = (torch.randn(N, kin2, device=dev, generator=g) / 12).to(torch.bfloat16)
        l2w, l2b = torch.randn(kin2, device=dev, generator=g), torch.randn(kin2, device=dev, generator=g)
        _, m2, s2 = K.ln_linear_fwd(X2, l2w, l2b, 1e-5, w2, bias, 0, None, True, True)
        sz2 = [kin2, kin2, N * kin2, N]
        pd2 = [(n + 3) // 4 * 4 for n in sz2]
        of2 = [sum(pd2[:i]) for i in range(4)]
        sl2 = torch.empty(nt, sum(pd2), device=dev)
        v2 = [sl2[:, o:o + n] for o, n in zip(of2, sz2)]
        res[f"ln_linear_bwd slab dense Kin={kin2}"] = timeit(
            lambda: K.ln_linear_bwd(G, w2, X2, m2, s2, l2w, l2b, None, False, v2[0], v2[1], v2[2], v2[3], slab=True))


if __name__ == "__main__":
    main()
