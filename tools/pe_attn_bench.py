"""Micro-benchmark of the implicit-K/V encoder cross-attention kernels at the ImageNet shape
(B = 32, M = 224·224, Nq = 32, H = 4, nc = 3): forward (attn_fwd_pe + combine) and backward
(attn_bwd_pe_implicit, per-sample queries), for kernel traces and PMC passes.
    python tools/pe_attn_bench.py [--iters N] [--which fwd|bwd|both]"""
import argparse
import math
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--which", default="both")
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--det", action="store_true", help="deterministic mode: per-key-block dQ slices, no atomics")
    a = ap.parse_args()
    from perceiver_io_amd.ops import emulation, ext

    K = ext.require()
    if a.det:
        K.set_deterministic(True)
    torch.manual_seed(0)
    B, M, Nq, H, nc, kin = a.B, 224 * 224, 32, 4, 3, 133
    C = 32 * H
    dev = "cuda"
    E = torch.rand(M, kin - nc, device=dev) * 2 - 1
    W = torch.randn(2 * C, kin, device=dev) / math.sqrt(kin)
    g, b = 1 + 0.1 * torch.randn(kin, device=dev), 0.1 * torch.randn(kin, device=dev)
    bias = 0.1 * torch.randn(2 * C, device=dev)
    Kp = -(-kin // 32) * 32
    Ebf = torch.zeros(M, Kp, device=dev)
    Ebf[:, nc:kin] = E
    Ebf = Ebf.to(torch.bfloat16)
    wg, _, _, _, wt = K.pe_weight_prep(W, g, b, bias, nc, Kp)
    P = K.pe_gemm(Ebf, wg, bf16_out=True, pad_rows=64)
    pes, pesq = E.sum(1).contiguous(), (E * E).sum(1).contiguous()
    pix = torch.randn(B * M, nc, device=dev)
    q = torch.randn(B, Nq, C, device=dev).to(torch.bfloat16)
    dO = torch.randn(B, Nq, C, device=dev).to(torch.bfloat16)
    scale = 1 / math.sqrt(32)
    o, lse = K.attn_fwd_pe(q, P, pix, pes, pesq, wt, H, scale, kin, 1e-5, 0)
    delta = (dO.float().view(B, Nq, H, 32) * o.float().view(B, Nq, H, 32)).sum(-1).contiguous()
    nkb = (M + 255) // 256
    dq = torch.empty(B, Nq, C, device=dev)
    D = torch.empty(M, 2 * C, device=dev)
    part = torch.empty(K.attn_bwd_pe_part_rows(M, H, B, 1), (2 + nc) * 2 * C, device=dev)
    for which in (("fwd", "bwd") if a.which == "both" else (a.which,)):
        def run():
            if which == "fwd":
                K.attn_fwd_pe(q, P, pix, pes, pesq, wt, H, scale, kin, 1e-5, 0)
            else:
                K.attn_bwd_pe_implicit(q, P, pes, pesq, wt, dO, lse, delta, pix, dq, D, part, H, scale, kin, 1e-5,
                                       False, 1)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
        print(f"{which}: {(time.perf_counter() - t0) / a.iters * 1e6:.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
