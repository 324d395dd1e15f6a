"""Is the latent self-attention backward latency-bound per workgroup?  Times attn_bwd at the
headline shape (N = 256, H = 4, D = 16) for B = 64 on one stream, B = 32 on one stream, and two
B = 32 halves on two streams at once (each variant captured in one hipGraph of `reps` launches,
so host launch cost is out of the picture).

    python tools/concurrency_probe.py
"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from perceiver_io_amd.ops import ext

    K = ext.require()
    H, D, N = 4, 16, 256
    C = H * D
    sc = 1 / math.sqrt(D)
    reps = 20

    def make(B):
        qkv = torch.randn(B, N, 3 * C, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
        o, lse = K.attn_fwd(q, k, v, None, H, D, sc, 0.0, None, 1)
        do = torch.randn(B, N, C, device="cuda").to(torch.bfloat16)
        delta = (do.float() * o.float()).view(B, N, H, D).sum(-1).contiguous()
        d = torch.empty(B, N, 3 * C, device="cuda")
        fwd = lambda: K.attn_fwd(q, k, v, None, H, D, sc, 0.0, None, 1)  # noqa: E731
        bwd = lambda: K.attn_bwd(q, k, v, None, o, do, lse, delta, H, D, sc, 0.0, None,  # noqa: E731
                                 d[:, :, :C], d[:, :, C:2 * C], d[:, :, 2 * C:])
        return fwd, bwd

    def timed_graph(body):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()  # warm-up (allocations) outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / 10 * 1e3 / reps

    for which in (0, 1):
        name = ("fwd", "bwd")[which]
        f64 = make(64)[which]
        f32a, f32b = make(32)[which], make(32)[which]
        t64 = timed_graph(lambda: [f64() for _ in range(reps)])
        t32 = timed_graph(lambda: [f32a() for _ in range(reps)])

        def two():
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            for _ in range(reps):
                f32a()
            with torch.cuda.stream(side):
                for _ in range(reps):
                    f32b()
            cur.wait_stream(side)
        t2 = timed_graph(two)
        print(f"attn_{name}: B=64 one stream {t64:6.2f} us | B=32 one stream {t32:6.2f} us | "
              f"2 x B=32 on two streams {t2:6.2f} us per pair", flush=True)


if __name__ == "__main__":
    main()
