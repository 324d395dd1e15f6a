"""Per-kernel dispatch cost of a replayed hipGraph of dependent tiny kernels.

Every MLM step replays ~120 dependent kernels; rocprof shows a ~4 µs floor even for a
256-thread fill, so the dispatch chain itself is a first-order cost.  This measures that
floor (µs per kernel = graph replay time / kernels) under runtime settings passed as
KEY=VALUE arguments, each configuration in its own child process:

    python tools/launch_overhead.py                       # default + a sweep of settings
    python tools/launch_overhead.py --child HIP_FORCE_DEV_KERNARG=1
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

SWEEP = [
    {},
    {"HIP_FORCE_DEV_KERNARG": "1"},
    {"HIP_FORCE_DEV_KERNARG": "0"},
    {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"},
    {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"},
    {"DEBUG_HIP_GRAPH_BATCH_SIZE": "1024"},
    {"AMD_DIRECT_DISPATCH": "0"},
]


def child(n_kernels: int = 200, reps: int = 50) -> dict:
    import torch
    dev = torch.device("cuda")
    out = {}
    for numel in (256, 1 << 20):
        x = torch.zeros(numel, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n_kernels):
                x.add_(1.0)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[f"graph_us_per_kernel_numel{numel}"] = e0.elapsed_time(e1) * 1e3 / (reps * n_kernels)
        # plain stream launches
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps * 10):
            x.add_(1.0)
        e1.record()
        torch.cuda.synchronize()
        out[f"stream_us_per_kernel_numel{numel}"] = e0.elapsed_time(e1) * 1e3 / (reps * 10)
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        for kv in sys.argv[2:]:
            k, v = kv.split("=", 1)
            assert os.environ.get(k) == v, f"{k} must be set before the runtime loads"
        print(json.dumps(child()), flush=True)
        return
    for cfg in SWEEP:
        env = dict(os.environ, **cfg)
        args = [sys.executable, __file__, "--child"] + [f"{k}={v}" for k, v in cfg.items()]
        r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
        res = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-400:]
        print(json.dumps({"env": cfg, "result": res}), flush=True)


if __name__ == "__main__":
    main()
