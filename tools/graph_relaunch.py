"""Does re-launching the SAME hipGraph exec serialise the host against the previous launch?

Captures a chain of small kernels (~100 nodes, like the training step) and times K replays of
one graph vs alternating between two captured copies, plus the host time spent inside
``replay()``.  Prints one JSON line per mode.

    python tools/graph_relaunch.py [--nodes 114] [--reps 200]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=114)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--numel", type=int, default=1 << 20)
    ap.add_argument("--busy-us", type=float, default=0.0, help="host work after each replay")
    a = ap.parse_args()
    dev = torch.device("cuda")
    s = torch.cuda.Stream()
    x = torch.randn(a.numel, device=dev)

    def body():
        y = x
        for _ in range(a.nodes):
            y = y.mul_(1.0000001)
        return y

    graphs = []
    with torch.cuda.stream(s):
        body()
        torch.cuda.synchronize()
        for _ in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                body()
            graphs.append(g)
    torch.cuda.synchronize()
    for mode in ("same", "alternate", "same", "alternate"):
        with torch.cuda.stream(s):
            for i in range(10):
                graphs[i % 2 if mode == "alternate" else 0].replay()
            torch.cuda.synchronize()
            host = 0.0
            t0 = time.perf_counter()
            for i in range(a.reps):
                h0 = time.perf_counter()
                graphs[i % 2 if mode == "alternate" else 0].replay()
                host += time.perf_counter() - h0
                if a.busy_us:
                    t1 = time.perf_counter() + a.busy_us * 1e-6
                    while time.perf_counter() < t1:
                        pass
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        print(json.dumps({"mode": mode, "nodes": a.nodes, "us_per_replay": dt / a.reps * 1e6,
                          "host_us_in_replay": host / a.reps * 1e6, "busy_us": a.busy_us}), flush=True)


if __name__ == "__main__":
    main()
