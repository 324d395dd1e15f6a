#!/usr/bin/env python
"""Headline benchmark: IMDB masked-language-model training throughput (samples/s, whole job).

Config (BASELINE.json config 2 / metric): Perceiver IO MLM, seq_len 512, vocab 10003,
256 latents × 64 channels, 3 encoder layers × (1 cross + 6 self-attention), 4/4/4 heads,
dropout 0, batch 64 per GPU (reference README MLM command), AdamW + OneCycleLR, bf16 compute.
Synthetic token ids of that shape, random-init weights (no network on the GPU box).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL)

Prints ONE JSON line on rank 0.  ``--backend reference`` measures the reference's own
compute (nn.MultiheadAttention math, full-logit CE, torch AdamW) eagerly on the same
device — the bar recorded in BASELINE.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_FILE = os.path.join(ROOT, "bench", "baseline_measured.json")


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Perceiver IO MLM training throughput")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch (reference README: 64)")
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--latents", type=int, default=256)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--vocab", type=int, default=10003)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch", "reference"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture of the step")
    ap.add_argument("--profile-steps", type=int, default=0)
    return ap.parse_args(argv)


def build(args, device):
    import torch

    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    lit = LitMaskedLanguageModel(
        vocab_size=args.vocab, max_seq_len=args.seq_len,
        optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 3e-3, "weight_decay": 0.0}},
        scheduler_init={"class_path": "torch.optim.lr_scheduler.OneCycleLR",
                        "init_args": {"max_lr": 3e-3, "total_steps": 50000, "pct_start": 0.1, "cycle_momentum": False}},
        num_latents=args.latents, num_latent_channels=args.channels, num_encoder_layers=3,
        num_encoder_cross_attention_heads=4, num_encoder_self_attention_heads=4,
        num_encoder_self_attention_layers_per_block=6, num_decoder_cross_attention_heads=4, dropout=0.0,
        masked_samples=None)
    lit.to(device)
    return lit


def main(argv=None):
    args = parse(argv)
    import torch

    from perceiver_io_amd import ops
    from perceiver_io_amd.parallel import FlatGradReducer, dist as pdist
    from perceiver_io_amd.train.engine import StepEngine

    info = pdist.init()
    world = info.world_size
    if world != args.gpus and pdist.env_world_size() > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    ops.set_backend("auto" if args.backend == "hip" else args.backend)
    torch.manual_seed(1234 + info.rank)

    lit = build(args, device)
    model = lit.model
    B, L = args.batch, args.seq_len
    fused = args.backend == "hip" and cuda
    if fused:
        from perceiver_io_amd.ops.optim import FusedAdamW

        opt = FusedAdamW(model.parameters(), lr=3e-3, weight_decay=0.0)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=3e-3, weight_decay=0.0)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=3e-3, total_steps=50000, pct_start=0.1,
                                                cycle_momentum=False)
    reducer = None
    if world > 1:
        from perceiver_io_amd.ops.optim import FlatParameterSpace

        flat = opt.flat if fused else FlatParameterSpace(model.parameters(), with_shadow=False)
        reducer = FlatGradReducer(flat, bucket_bytes=64 << 20)
        reducer.broadcast_parameters(model)

    autocast = (not fused) and args.dtype == "bf16" and cuda

    def loss_fn(batch):
        _, ids, pad = batch
        if autocast:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return model.loss(ids, pad)
        return model.loss(ids, pad)

    engine = StepEngine(loss_fn, opt, sched, reducer=reducer, device=device, graph=fused and not args.no_graph)
    g = torch.Generator(device="cpu").manual_seed(99 + info.rank)

    def batch():
        ids = torch.randint(3, args.vocab, (B, L), generator=g)
        pad = torch.zeros(B, L, dtype=torch.bool)
        return (torch.zeros(B, dtype=torch.long), ids.to(device), pad.to(device))

    data = [batch() for _ in range(4)]
    for i in range(args.warmup):
        loss = engine.step(data[i % 4])
    if cuda:
        torch.cuda.synchronize()
    pdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = engine.step(data[i % 4])
    if cuda:
        torch.cuda.synchronize()
    pdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = pdist.all_reduce_max(dt)
    final_loss = float(loss.float().item())
    if args.profile_steps and cuda:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(args.profile_steps):
                engine.step(data[i % 4])
            torch.cuda.synchronize()
        if info.is_main:
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40), file=sys.stderr)
    ms = dt / args.steps * 1e3
    value = B * world * args.steps / dt
    # bar: the reference's own compute measured eagerly on one MI355X (bench/baseline_measured.json,
    # recorded in BASELINE.md); weak scaling → compare against world × per-GPU reference rate
    vs = None
    if os.path.exists(BASELINE_FILE):
        try:
            ref = float(json.load(open(BASELINE_FILE))["mlm256_reference_samples_per_s_per_gpu"])
            vs = value / (ref * world)
        except Exception:
            vs = None
    if info.is_main:
        out = {
            "metric": "samples/sec (whole node) IMDB MLM seq_len=512 at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(vs, 3) if vs else None,
            "dtype": args.dtype if not fused else "bf16", "data": "synthetic (random token ids, random-init weights)",
            "config": {"model": f"perceiver-io-mlm latents={args.latents}x{args.channels} layers=3x(1+6) vocab={args.vocab}",
                       "global_batch": B * world, "seq_len": L, "parallelism": f"dp{world}",
                       "backend": args.backend, "graph": bool(fused and not args.no_graph)},
            "final_loss": round(final_loss, 4),
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
