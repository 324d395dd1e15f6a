"""A/B timing of the headline's latent self-attention backward (B = 64, N = 256, C = 64, H = 4,
bf16 dQ/dK/dV) with and without the carried slab reduction, and with slabs of half the rows
(the read traffic a bf16 slab would have), to price the slab traffic on the critical path.

    python tools/slab_ab.py [--reps 200]
"""
import argparse
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--cols", type=int, default=24960, help="slab row length (one layer's parameters)")
    args = ap.parse_args()
    from perceiver_io_amd.ops import ext

    K = ext.require()
    dev = "cuda"
    B, N, H, D = 64, 256, 4, 16
    E = H * D
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, N, 3 * E, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, :E], qkv[:, :, E:2 * E], qkv[:, :, 2 * E:]
    do = torch.randn(B, N, E, device=dev, generator=g).to(torch.bfloat16)
    o, lse = K.attn_fwd(q, k, v, None, H, D, scale, 0.0, None, 1)
    delta = (do.float().view(B, N, H, D) * o.float().view(B, N, H, D)).sum(-1).contiguous()
    dqkv = torch.empty(B, N, 3 * E, device=dev, dtype=torch.bfloat16)
    out = {}
    for rows in (0, 64, 128, 256):
        job = {}
        if rows:
            slab = torch.randn(rows, args.cols + 64, device=dev, generator=g)
            dst = torch.zeros(args.cols, device=dev)
            job = dict(job_slab=slab, job_dsts=[dst], job_offs=[0])

        def run():
            K.attn_bwd(q, k, v, None, o, do, lse, delta, H, D, scale, 0.0, None, dqkv[:, :, :E], dqkv[:, :, E:2 * E],
                       dqkv[:, :, 2 * E:], **job)

        for _ in range(20):
            run()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(args.reps):
            run()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1e3 / args.reps
        out[f"slab_rows_{rows}"] = round(us, 2)
        print(f"attn_bwd bf16 + slab {rows:3d} x {args.cols}: {us:7.2f} us / launch", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
