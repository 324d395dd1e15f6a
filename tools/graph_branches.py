"""Do forked-stream branches of a captured hipGraph run concurrently on this ROCm?

Captures two spin kernels (torch.cuda._sleep) either on one stream (serial) or on two streams
forked from / joined to the capture stream, and times replays of each graph.  Concurrent
branches: the forked graph takes ~max of the two, serial ~their sum.

    python tools/graph_branches.py [cycles]
"""
import sys
import time

import torch


def main():
    cyc = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    main_s = torch.cuda.Stream()
    side = torch.cuda.Stream()

    def body(fork):
        torch.cuda._sleep(cyc)
        if fork:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            torch.cuda._sleep(cyc)
            torch.cuda.current_stream().wait_stream(side)
        else:
            torch.cuda._sleep(cyc)
            torch.cuda._sleep(cyc)

    res = {}
    for fork in (False, True):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(main_s):
            body(fork)  # warm-up
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=main_s):
                body(fork)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        res[fork] = (time.perf_counter() - t0) / 10 * 1e6
    # eager two-stream reference
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        body(True)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 10 * 1e6
    print(f"serial graph {res[False]:.1f} us, forked graph {res[True]:.1f} us, eager forked {eager:.1f} us "
          f"(3 sleeps; concurrent branches => forked ~ 2/3 of serial)")


if __name__ == "__main__":
    main()
