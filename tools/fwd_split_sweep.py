"""Split-KV sweep of the attention forward (attn_fwd + combine) at the configs' cross-attention
shapes, against ops.attention.pick_splits' choice.

    python tools/fwd_split_sweep.py
"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.microbench import timeit  # noqa: E402


def main():
    from perceiver_io_amd.ops import ext
    from perceiver_io_amd.ops.attention import pick_splits

    K = ext.require()
    H, D = 4, 16
    C = H * D
    shapes = [("mlm256 enc cross", 64, 256, 512, 0.0), ("mlm64 enc cross", 64, 64, 512, 0.0),
              ("seq_clf enc cross", 128, 64, 512, 0.0), ("seq_clf_ft enc cross", 128, 64, 512, 0.1),
              ("long_mlm enc cross", 8, 512, 8192, 0.0), ("mlm256 dec cross", 64, 77, 256, 0.0),
              ("lartpc-like 4k keys", 4, 32, 4096, 0.0), ("lartpc-like 8k keys", 4, 32, 8192, 0.0),
              ("lartpc-like 16k keys", 4, 32, 16384, 0.0)]
    seed = torch.zeros(1, dtype=torch.int64, device="cuda")
    for name, B, Nq, Nk, p in shapes:
        q = torch.randn(B, Nq, C, device="cuda").to(torch.bfloat16)
        kv = torch.randn(B, Nk, 2 * C, device="cuda").to(torch.bfloat16)
        k, v = kv[:, :, :C], kv[:, :, C:]
        sc = 1 / math.sqrt(D)
        pick = pick_splits(B, H, Nq, Nk, p > 0)
        row = []
        for ns in (1, 2, 4, 8, 16, 32, 64):
            if ns > (Nk + 63) // 64:
                continue
            t = timeit(lambda: K.attn_fwd(q, k, v, None, H, D, sc, p, seed if p > 0 else None, ns), iters=100)
            row.append(f"{ns}:{t:6.1f}")
        print(f"{name:22s} B={B:4d} Nq={Nq:4d} Nk={Nk:5d} p={p}  pick={pick}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
