"""Time the fused layer kernels at the headline shape (B=64, N=256, C=64): run once with
PIO_CHAIN=1 (register-resident chain kernels) and once with PIO_CHAIN=0 (LDS row-pass kernels).

    PIO_CHAIN=1 python tools/chain_bench.py ; PIO_CHAIN=0 python tools/chain_bench.py   (GPU)
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from perceiver_io_amd.ops import ext  # noqa: E402
from tools.microbench import timeit  # noqa: E402


def main():
    K = ext.require()
    dev, bf = "cuda", torch.bfloat16
    B, N, C = 64, 256, 64
    R = B * N
    torch.manual_seed(0)
    qkv = torch.randn(R, 3 * C, device=dev).to(bf)
    x = torch.randn(R, C, device=dev)

    def w(*s):
        return (torch.randn(*s, device=dev) * 0.15).to(bf)

    wo, w1, w2, wq = w(C, C), w(C, C), w(C, C), w(3 * C, C)
    v = [torch.randn(C, device=dev) * 0.1 for _ in range(7)]
    bq = torch.randn(3 * C, device=dev) * 0.1
    args = (qkv, x, N, 0.25, wo, v[0], v[1], v[2], 1e-5, w1, v[3], w2, v[4])
    t_next = timeit(lambda: K.sa_layer_fwd(*args, lnw=v[5], lnb=v[6], wq=wq, bq=bq))
    t_last = timeit(lambda: K.sa_layer_fwd(*args))
    print(f"PIO_CHAIN={os.environ.get('PIO_CHAIN', '1')} sa_layer_fwd next={t_next:.2f} us last={t_last:.2f} us")


if __name__ == "__main__":
    main()
