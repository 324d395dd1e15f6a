#!/usr/bin/env python
"""LArTPC per-pixel semantic segmentation with Perceiver IO (reference ``run.py``).

512×512 single-plane wire images → 3 classes per pixel (background / track / shower).  The
model is the reference's (``perceiver_io_amd/models/lartpc.py``): Fourier-encoded image input,
32×64 latents, 3 layers × (1 cross + 3 self-attention), one decoder query per pixel, a 3-way
classifier, and a U-ResNet built alongside (unused, as in the reference).  Training follows
the reference: weighted cross-entropy with background weight 0, Adam (lr 1e-3, L2 weight decay
1e-4), grad-norm clip 10, ReduceLROnPlateau(patience 5000, factor 0.1) stepped on the training
loss, batch 4, per-class accuracies, validation each epoch, and a checkpoint
``{'epoch', 'model_state_dict', 'optimizer_state_dict'}``.

On a GPU the default is the MI355X path:

* **sparse execution** (``models/lartpc.py``).  The encoder sees only the non-zero pixels and
  the decoder only the weighted pixels.  Loss and gradients are the same as the dense model's.
  Pass ``--dense`` to run all 262,144 keys and queries, the reference's cost.
* **fused kernels + hipGraph step** (``StepEngine``).  One graph is captured per capacity bucket.
  ``FusedAdam`` does the coupled-L2 Adam update and the clip in one kernel pass.
  ReduceLROnPlateau reads the previous step's loss, so the host never waits on the step in
  flight.  The reference steps it on the current loss; with patience 5000 the one-step lag
  changes nothing in practice.

``--engine eager`` (the default on CPU) runs the reference sequence exactly: zero_grad,
forward, ``scheduler.step(loss)``, backward, ``clip_grad_norm_``, ``Adam.step``.

Documented differences: a synthetic track/shower generator stands in for the larcv/ROOT
reader (``data/synthetic.py:lartpc_event``), because larcv and ROOT are not available.
Logits are permuted to (B, 3, H·W) instead of reshaped (defect D6).  Metrics go to
tfevents/JSONL.  With the fused optimizer, ``optimizer_state_dict`` covers the trained (Perceiver)
parameters.  The unused U-ResNet never has a gradient, and torch's Adam skips it too.

    python run.py [--epochs 10] [--events 64] [--size 512] [--batch-size 4] [--dense] [--engine eager]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from perceiver_io_amd.data.lartpc import SparseCollator  # noqa: E402
from perceiver_io_amd.data.synthetic import SyntheticLArTPC  # noqa: E402
from perceiver_io_amd.models.lartpc import LArPerceiver, accuracies, class_weights  # noqa: E402
from perceiver_io_amd.train.loggers import TensorBoardLogger  # noqa: E402

__all__ = ["LArPerceiver", "accuracies", "main"]


def _to(batch, dev):
    return tuple(t.to(dev, non_blocking=True) for t in batch)


def make_step_fn(model, weights, sparse: bool, metrics: dict):
    """loss_fn(batch) → loss; per-class accuracies of the batch land in ``metrics`` (device)."""

    def loss_fn(batch):
        if sparse:
            loss, acc = model.sparse_loss(batch, weights)
        else:
            img, lab = batch
            out = model(img)
            loss = F.cross_entropy(out, lab, weight=weights)
            acc = accuracies(out.argmax(1).detach(), lab)
        metrics.update(acc)
        return loss

    return loss_fn


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--events", type=int, default=64)
    ap.add_argument("--val-events", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--max-steps", type=int, default=-1)
    ap.add_argument("--log-dir", default="runs")
    ap.add_argument("--ckpt-dir", default="ckpt")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--engine", choices=["auto", "graph", "eager"], default="auto",
                    help="graph: fused kernels + hipGraph step (GPU default); eager: the reference sequence")
    ap.add_argument("--dense", action="store_true", help="evaluate all pixels (the reference's cost)")
    ap.add_argument("--bucket", type=int, default=2048, help="sparse capacity rounding (keys / queries)")
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--workers", type=int, default=1)
    a = ap.parse_args(argv)
    dev = torch.device(a.device)
    torch.manual_seed(0)
    model = LArPerceiver(a.size).to(dev)
    weights = class_weights(dev)
    sparse = not a.dense
    collate = SparseCollator(a.bucket) if sparse else None
    kw = dict(num_workers=a.workers, persistent_workers=a.workers > 0, collate_fn=collate)
    train = torch.utils.data.DataLoader(SyntheticLArTPC(a.events, a.size, seed=0), batch_size=a.batch_size,
                                        shuffle=True, drop_last=True, **kw)
    val = torch.utils.data.DataLoader(SyntheticLArTPC(a.val_events, a.size, seed=1), batch_size=a.batch_size,
                                      drop_last=True, collate_fn=collate)
    fused = dev.type == "cuda" and a.engine != "eager"
    if fused:
        from perceiver_io_amd.ops.optim import FusedAdam
        from perceiver_io_amd.train.engine import StepEngine

        opt = FusedAdam(model.trained_parameters(), lr=a.lr, weight_decay=1e-4, max_grad_norm=10.0)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=a.lr, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, patience=5000, factor=0.1)
    metrics: dict = {}
    loss_fn = make_step_fn(model, weights, sparse, metrics)
    engine = None
    if fused:
        engine = StepEngine(loss_fn, opt, None, device=dev, graph=True,
                            state_hooks=(lambda: dict(metrics), lambda s: metrics.update(s)))
    log = TensorBoardLogger(a.log_dir, name="lartpc")
    step, epoch, prev = 0, 0, None
    t_start, n_timed = None, 0
    for epoch in range(a.epochs):
        model.train()
        for batch in train:
            batch = _to(batch, dev)
            t0 = time.perf_counter()
            if fused:
                loss = engine.step(batch)
                if prev is not None:
                    sched.step(float(prev))  # the previous step's loss: no wait on this one
                prev = loss
            else:
                opt.zero_grad()
                loss = loss_fn(batch)
                sched.step(loss.item())  # stepped before backward, like the reference
                loss.backward()
                torch.nn.utils.clip_grad_norm_(model.parameters(), 10)
                opt.step()
            if step == 2:  # throughput after graph capture / allocator warm-up
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t_start, n_timed = time.perf_counter(), 0
            elif t_start is not None:
                n_timed += a.batch_size
            if step % a.log_every == 0:
                vals = {k: float(v) for k, v in metrics.items()}
                log.log_metrics({"loss": float(loss), "lr": opt.param_groups[0]["lr"],
                                 **{f"train_{k}": v for k, v in vals.items()}}, step)
                print(f"epoch {epoch} step {step} loss {float(loss):.4f} acc {vals.get('acc', 0):.3f} "
                      f"{time.perf_counter() - t0:.3f}s", flush=True)
            step += 1
            if 0 < a.max_steps <= step:
                break
        model.eval()
        vl, va = [], []
        with torch.no_grad():
            for batch in val:
                batch = _to(batch, dev)
                vm: dict = {}
                vl.append(float(make_step_fn(model, weights, sparse, vm)(batch)))
                va.append(float(vm["acc"]))
        if vl:
            log.log_metrics({"validation_loss": sum(vl) / len(vl), "val_acc": sum(va) / len(va)}, step)
            print(f"validation loss: {sum(vl) / len(vl):.4f}", flush=True)
        if 0 < a.max_steps <= step:
            break
    if t_start is not None and n_timed:
        if dev.type == "cuda":
            torch.cuda.synchronize()
        print(f"throughput: {n_timed / (time.perf_counter() - t_start):.1f} samples/s "
              f"({'sparse' if sparse else 'dense'}, {'fused graph' if fused else 'eager'})", flush=True)
    os.makedirs(a.ckpt_dir, exist_ok=True)
    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": opt.state_dict()},
               os.path.join(a.ckpt_dir, f"model_{epoch}.ckpt"))
    log.close()


if __name__ == "__main__":
    main()
