"""Split sweep of the factored Fourier-PE cross-attention forward (attn_fwd_pe + combine) at the
image configs' shapes, against the launcher's automatic choice (nsplit = 0).

    python tools/pe_fwd_split_sweep.py
"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.microbench import timeit  # noqa: E402


def main():
    from perceiver_io_amd.ops import ext

    K = ext.require()
    torch.manual_seed(0)
    dev = "cuda"
    H, Nq = 4, 32
    C = 32 * H
    for name, B, side, nc in (("mnist", 128, 28, 1), ("imagenet", 32, 224, 3)):
        M = side * side
        kin = nc + 2 * (2 * 32 + 1)
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
        sc = 1 / math.sqrt(32)
        row = []
        for ns in (0, 1, 2, 4, 8, 16, 32):
            t = timeit(lambda: K.attn_fwd_pe(q, P, pix, pes, pesq, wt, H, sc, kin, 1e-5, ns), iters=50)
            row.append(f"{ns if ns else 'auto'}:{t:6.1f}")
        print(f"{name:9s} B={B:4d} M={M:6d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
