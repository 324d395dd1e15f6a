"""Attention kernel timing vs batch (latency- vs throughput-bound diagnosis)."""
import math
import sys

import torch

sys.path.insert(0, ".")
from perceiver_io_amd.ops import ext  # noqa: E402
from tools.microbench import timeit  # noqa: E402


def main():
    K = ext.require()
    H, D, N = 4, 16, 256
    C = H * D
    batches = [int(a) for a in sys.argv[1:]] or [1, 8, 64, 256]
    for B in batches:
        qkv = torch.randn(B, N, 3 * C, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
        sc = 1 / math.sqrt(D)
        tf = timeit(lambda: K.attn_fwd(q, k, v, None, H, D, sc, 0.0, None, 1), iters=100)
        o, lse = K.attn_fwd(q, k, v, None, H, D, sc, 0.0, None, 1)
        do = torch.randn(B, N, C, device="cuda").to(torch.bfloat16)
        delta = (do.float() * o.float()).view(B, N, H, D).sum(-1).contiguous()
        d = torch.empty(B, N, 3 * C, device="cuda")
        tb = timeit(lambda: K.attn_bwd(q, k, v, None, o, do, lse, delta, H, D, sc, 0.0, None, d[:, :, :C], d[:, :, C:2 * C],
                                       d[:, :, 2 * C:]), iters=100)
        print(f"B={B:4d}  fwd {tf:8.2f} us   bwd {tb:8.2f} us")


if __name__ == "__main__":
    main()
