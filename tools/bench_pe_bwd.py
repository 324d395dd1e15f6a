"""Microbenchmark of the fused PE cross-attention backward (csrc/attention_pe.hip) at the
ImageNet-shape config (B = 32, M = 50,176, 32 latent queries, C = 128, 4 heads), with the old
attn_bwd (fp32 dK/dV) path and the forward for comparison.

    python tools/bench_pe_bwd.py [--B 32] [--M 50176]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--M", type=int, default=50176)
    ap.add_argument("--H", type=int, default=4)
    a = ap.parse_args()
    from perceiver_io_amd.ops import ext

    K = ext.require()
    B, M, H, Nq, nc = a.B, a.M, a.H, 32, 3
    C = 32 * H
    dev = "cuda"
    q = torch.randn(1, Nq, 3 * C, device=dev).bfloat16()[:, :, :C]
    kv = torch.randn(B * M, 2 * C, device=dev).bfloat16()
    dO = torch.randn(B, Nq, C, device=dev).bfloat16()
    scale = 1 / math.sqrt(32)
    kv3 = kv.view(B, M, 2 * C)
    o, lse = K.attn_fwd(q, kv3[:, :, :C], kv3[:, :, C:], None, H, 32, scale, 0.0, None, 8)
    delta = (dO.float().view(B, Nq, H, 32) * o.float().view(B, Nq, H, 32)).sum(-1).contiguous()
    pix = torch.randn(B * M, nc, device=dev)
    mean = torch.randn(B * M, device=dev) * 0.1
    rstd = torch.rand(B * M, device=dev) + 0.5
    nkb = (M + 255) // 256
    dq = torch.empty(Nq, C, device=dev)
    D = torch.empty(M, 2 * C, device=dev)
    part = torch.empty(nkb, (2 + nc) * 2 * C, device=dev)
    gb = kv.numel() * 2 / 1e9
    us = timeit(lambda: K.attn_bwd_pe(q, kv, dO, lse, delta, mean, rstd, pix, dq, D, part, H, scale, False, 1))
    print(f"attn_bwd_pe (broadcast queries): {us:8.1f} us   (K/V {gb:.2f} GB → {gb / us * 1e3:.2f} TB/s)")
    qb = torch.randn(B, Nq, 3 * C, device=dev).bfloat16()[:, :, :C]
    dqb = torch.empty(B, Nq, C, device=dev)
    us = timeit(lambda: K.attn_bwd_pe(qb, kv, dO, lse, delta, mean, rstd, pix, dqb, D, part, H, scale, False, 1))
    print(f"attn_bwd_pe (per-sample queries): {us:8.1f} us   (K/V {gb:.2f} GB → {gb / us * 1e3:.2f} TB/s)")
    dkv = torch.empty(B, M, 2 * C, device=dev)

    def old():
        K.attn_bwd(q, kv3[:, :, :C], kv3[:, :, C:], None, o, dO, lse, delta, H, 32, scale, 0.0, None, None,
                   dkv[:, :, :C], dkv[:, :, C:], False)
    print(f"attn_bwd (writes fp32 dK/dV): {timeit(old):8.1f} us")
    print(f"attn_fwd (split 8):           {timeit(lambda: K.attn_fwd(q, kv3[:, :, :C], kv3[:, :, C:], None, H, 32, scale, 0.0, None, 8)):8.1f} us")


if __name__ == "__main__":
    main()
