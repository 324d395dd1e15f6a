"""Step-by-step diagnosis of the MLM training step (bench.py's headline config): eager steps,
then captured-graph replays, each followed by a device sync, a finite-loss check and the
persistent kernels' error word (csrc/persist.hip).  python tools/persist_diag.py [--graph-steps N]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from perceiver_io_amd.ops import ext  # noqa: E402
from perceiver_io_amd.ops.optim import FusedAdamW  # noqa: E402
from perceiver_io_amd.train.engine import StepEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eager-steps", type=int, default=6)
    ap.add_argument("--graph-steps", type=int, default=40)
    ap.add_argument("--config", default="mlm256")
    a = ap.parse_args()
    args = bench.parse(["--config", a.config])
    dev = torch.device("cuda:0")
    K = ext.require()
    lit, loss_fn, make_batch, desc, lr, wd = bench.build(args, dev)
    lit.to(dev)
    params = [p for p in lit.model.parameters() if p.requires_grad]
    g = torch.Generator(device="cpu").manual_seed(7)
    data = [tuple(t.to(dev) for t in make_batch(g)) for _ in range(4)]
    for graph, n in ((False, a.eager_steps), (True, a.graph_steps)):
        opt = FusedAdamW(params, lr=lr, weight_decay=wd)
        eng = StepEngine(loss_fn, opt, None, device=dev, graph=graph)
        K.persist_errors(True)
        for i in range(n):
            t = time.perf_counter()
            loss = eng.step(data[i % 4])
            torch.cuda.synchronize()
            err = K.persist_errors(True)
            lv = float(loss.float().item())
            print(f"graph={graph} step {i}: loss {lv:.4f} err {err} {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
            assert err == 0 and lv == lv, "persistent-kernel error or NaN loss"
    print("DIAG_OK")


if __name__ == "__main__":
    main()
