#!/usr/bin/env python
"""Training-throughput benchmark (samples/s, whole job) for the BASELINE.json configs.

Default (the headline, BASELINE.json metric / config 2): Perceiver IO MLM, seq_len 512,
vocab 10003, 256 latents × 64 channels, 3 encoder layers × (1 cross + 6 self-attention),
4/4/4 heads, dropout 0, batch 64 per GPU (reference README MLM command), AdamW + OneCycleLR,
bf16 compute.  Synthetic token ids of that shape, random-init weights (no network on the GPU box).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL)
    python bench.py --config {mlm256,mlm64,seq_clf,seq_clf_ft,imagenet,long_mlm,mnist,lartpc} ...

``mlm64`` = the reference README's MLM run itself (64 × 64 latents, batch 64, lr 3e-3).
Other configs (BASELINE.json configs 1, 3-5): ``seq_clf`` = IMDB text classifier with a frozen
encoder (decoder-only training, batch 128/GPU, README seq_clf command); ``imagenet`` =
224×224×3 image classifier with Fourier position encoding (50,176 inputs × 133 channels,
32×128 latents, 3×(1+3) layers, 1000 classes); ``long_mlm`` = MLM at seq_len 8192 with 512
latents; ``mnist`` = the 28×28 classifier of the README (batch 128); ``lartpc`` = the LArTPC
segmentation experiment of ``run.py`` (512×512 synthetic events, batch 4, Adam + clip 10; the
HIP backend runs it sparse — loss and gradients equal to the dense model's, see
``models/lartpc.py`` — and ``--backend reference`` densely, as the reference does).

Prints ONE JSON line on rank 0.  ``--backend reference`` measures the reference's own compute
(nn.MultiheadAttention math, full-logit CE, torch AdamW) eagerly under bf16 autocast on the same
device — the bar recorded in BASELINE.md and bench/baseline_measured.json.
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
HEADLINE_METRIC = "samples/sec (whole node) IMDB MLM seq_len=512 at 1/2/4/8 MI355X"

# config name → defaults (batch per GPU, sequence length / inputs) and the metric string
CONFIGS = {
    "mlm256": dict(batch=64, seq_len=512, latents=256, channels=64, metric=HEADLINE_METRIC),
    # the reference README's own MLM run (README.md:33-44, scripts/mlm.py:19-29): 64 × 64 latents
    "mlm64": dict(batch=64, seq_len=512, latents=64, channels=64,
                  metric="samples/sec (whole node) IMDB MLM seq_len=512 64x64 latents (reference README run)"),
    "seq_clf": dict(batch=128, seq_len=512, latents=64, channels=64,
                    metric="samples/sec (whole node) IMDB seq_clf frozen encoder seq_len=512"),
    # the README's joint fine-tune (README.md:91-107): encoder unfrozen, dropout 0.1, lr 1e-4
    "seq_clf_ft": dict(batch=128, seq_len=512, latents=64, channels=64,
                       metric="samples/sec (whole node) IMDB seq_clf joint fine-tune dropout 0.1 seq_len=512"),
    "imagenet": dict(batch=32, seq_len=224 * 224, latents=32, channels=128,
                     metric="samples/sec (whole node) ImageNet-shape 224x224x3 img_clf Fourier PE"),
    "long_mlm": dict(batch=8, seq_len=8192, latents=512, channels=64,
                     metric="samples/sec (whole node) IMDB MLM seq_len=8192 512 latents"),
    "mnist": dict(batch=128, seq_len=28 * 28, latents=32, channels=128,
                  metric="samples/sec (whole node) MNIST img_clf 32x128 latents"),
    "lartpc": dict(batch=4, seq_len=512 * 512, latents=32, channels=64,
                   metric="samples/sec (whole node) LArTPC 512x512 per-pixel segmentation (run.py)"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Perceiver IO training throughput")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="mlm256", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--latents", type=int, default=None)
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=10003)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch", "reference"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture of the step")
    ap.add_argument("--allreduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce wire format (N > 1)")
    ap.add_argument("--overlap", default="off", choices=["on", "off"],
                    help="N > 1: bucket all-reduces at ready points on a side stream during the backward (on) or "
                         "one all-reduce after the backward on the compute stream (off, default)")
    ap.add_argument("--bucket-update", default="auto", choices=["auto", "on", "off"],
                    help="N > 1: AdamW per bucket right behind its all-reduce (on; auto = with --overlap on) or one "
                         "pass after all (off)")
    ap.add_argument("--dense", action="store_true", help="lartpc: evaluate all pixels (the reference's cost)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--profile-stacks", type=int, default=0,
                    help="with --profile-steps: list the framework (aten) ops that touch device tensors in the "
                         "profiled steps with N Python stack frames each (finds stray copies / fills)")
    a = ap.parse_args(argv)
    cfg = CONFIGS[a.config]
    for k in ("batch", "seq_len", "latents", "channels"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    return a


def _aten_stacks(engine, data, steps, depth):
    """Every aten op that touches a device tensor during `steps` eager steps, grouped by op and
    the innermost `depth` Python frames (a dispatch-mode hook: sees the ops issued from C++
    extension code and from the autograd threads too)."""
    import collections
    import traceback

    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch.utils._pytree import tree_flatten

    quiet = ("aten::view", "aten::_unsafe_view", "aten::slice", "aten::as_strided", "aten::empty", "aten::empty_strided",
             "aten::detach", "aten::alias", "aten::t", "aten::transpose", "aten::permute", "aten::expand",
             "aten::select", "aten::unsqueeze", "aten::squeeze", "aten::reshape", "aten::_reshape_alias",
             "aten::lift_fresh", "aten::set_", "aten::resize_", "aten::split", "aten::unbind", "aten::chunk",
             "aten::narrow", "aten::diagonal", "aten::new_empty", "aten::new_empty_strided", "aten::is_nonzero")
    seen = collections.Counter()

    class _Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = func._schema.name
            if name not in quiet:
                flat, _ = tree_flatten((args, kwargs or {}))
                if any(isinstance(t, torch.Tensor) and t.device.type == "cuda" for t in flat):
                    frames = traceback.extract_stack()[:-1][-depth:]
                    seen[(str(func), tuple(f"{f.filename.split('/repo/')[-1]}:{f.lineno} {f.name}" for f in frames))] += 1
            return out

    with _Rec():
        for i in range(steps):
            engine.step(data[i % 4], ring_view=True)
        torch.cuda.synchronize()
    for (op, frames), n in seen.most_common(60):
        print(f"{op} x{n}", file=sys.stderr)
        for fr in frames:
            print(f"    {fr}", file=sys.stderr)


def _opt(lr=3e-3, wd=0.0):
    return {"class_path": "torch.optim.AdamW", "init_args": {"lr": lr, "weight_decay": wd}}


def _sched(lr=3e-3):
    return {"class_path": "torch.optim.lr_scheduler.OneCycleLR",
            "init_args": {"max_lr": lr, "total_steps": 50000, "pct_start": 0.1, "cycle_momentum": False}}


def build(args, device):
    """→ (lit module, loss_fn(batch), make_batch(generator), model description, lr, weight decay)."""
    import torch

    from perceiver_io_amd.tasks import LitImageClassifier, LitMaskedLanguageModel, LitTextClassifier

    B, L = args.batch, args.seq_len
    if args.config == "lartpc":
        return _build_lartpc(args)
    if args.config in ("mlm256", "mlm64", "long_mlm"):
        lit = LitMaskedLanguageModel(
            vocab_size=args.vocab, max_seq_len=L, optimizer_init=_opt(), scheduler_init=_sched(),
            num_latents=args.latents, num_latent_channels=args.channels, num_encoder_layers=3,
            num_encoder_cross_attention_heads=4, num_encoder_self_attention_heads=4,
            num_encoder_self_attention_layers_per_block=6, num_decoder_cross_attention_heads=4, dropout=0.0,
            masked_samples=None)
        model = lit.model

        def loss_fn(batch):
            _, ids, pad = batch
            return model.loss(ids, pad)

        def make_batch(g):
            ids = torch.randint(3, args.vocab, (B, L), generator=g)
            return (torch.zeros(B, dtype=torch.long), ids, torch.zeros(B, L, dtype=torch.bool))

        desc = f"perceiver-io-mlm latents={args.latents}x{args.channels} layers=3x(1+6) vocab={args.vocab}"
        return lit, loss_fn, make_batch, desc, 3e-3, 0.0
    if args.config in ("seq_clf", "seq_clf_ft"):
        ft = args.config == "seq_clf_ft"
        lr, wd = (1e-4, 0.01) if ft else (1e-3, 0.01)
        lit = LitTextClassifier(
            num_classes=2, vocab_size=args.vocab, max_seq_len=L, freeze_encoder=not ft,
            optimizer_init=_opt(lr, wd), scheduler_init=None, num_latents=args.latents,
            num_latent_channels=args.channels, num_encoder_layers=3, num_encoder_cross_attention_heads=4,
            num_encoder_self_attention_heads=4, num_encoder_self_attention_layers_per_block=6,
            num_decoder_cross_attention_heads=1, dropout=0.1 if ft else 0.0)
        model = lit.model

        def loss_fn(batch):  # = cross_entropy(model(ids, pad), y); fused head on the HIP backend
            y, ids, pad = batch
            return model.loss(ids, y, pad)

        def make_batch(g):
            ids = torch.randint(3, args.vocab, (B, L), generator=g)
            return (torch.randint(0, 2, (B,), generator=g), ids, torch.zeros(B, L, dtype=torch.bool))

        desc = (f"perceiver-io-seq-clf {'joint-fine-tune dropout=0.1' if ft else 'frozen-encoder'} "
                f"latents={args.latents}x{args.channels} layers=3x(1+6) vocab={args.vocab}")
        return lit, loss_fn, make_batch, desc, lr, wd
    # image classifiers
    if args.config == "imagenet":
        side = int(round(args.seq_len ** 0.5))
        shape, classes, sa, bands = (side, side, 3), 1000, 3, 32
    else:
        shape, classes, sa, bands = (28, 28, 1), 10, 3, 32
    lit = LitImageClassifier(
        image_shape=shape, num_classes=classes, num_frequency_bands=bands, optimizer_init=_opt(1e-3, 0.01),
        scheduler_init=None, num_latents=args.latents, num_latent_channels=args.channels, num_encoder_layers=3,
        num_encoder_cross_attention_heads=4, num_encoder_self_attention_heads=4,
        num_encoder_self_attention_layers_per_block=sa, num_decoder_cross_attention_heads=1, dropout=0.0)
    model = lit.model

    def loss_fn(batch):  # = cross_entropy(model(x), y); fused head on the HIP backend
        x, y = batch
        return model.loss(x, y)

    def make_batch(g):
        return (torch.randn((B,) + shape, generator=g), torch.randint(0, classes, (B,), generator=g))

    desc = (f"perceiver-io-img-clf {shape[0]}x{shape[1]}x{shape[2]} fourier-bands={bands} "
            f"latents={args.latents}x{args.channels} layers=3x(1+{sa}) classes={classes}")
    return lit, loss_fn, make_batch, desc, 1e-3, 0.01


class _LArHolder:
    """``lit``-like holder: ``.model`` (with ``.decoder``), moved by ``.to``."""

    def __init__(self, model):
        self.model = model

    def to(self, device):
        self.model.to(device)
        return self


def _build_lartpc(args):
    import torch
    import torch.nn.functional as F

    from perceiver_io_amd.data.lartpc import sparse_collate
    from perceiver_io_amd.data.synthetic import lartpc_event
    from perceiver_io_amd.models.lartpc import LArPerceiver, class_weights

    side = int(round(args.seq_len ** 0.5))
    model = LArPerceiver(side, latents=(args.latents, args.channels))
    B = args.batch
    dense = args.backend == "reference" or args.dense
    state = {}

    def loss_fn(batch):
        w = state.get("w")
        if w is None or w.device != batch[0].device:
            w = state["w"] = class_weights(batch[0].device)
        if dense:
            img, lab = batch
            return F.cross_entropy(model(img).float(), lab, weight=w)
        return model.sparse_loss(batch, w)[0]

    pool = []

    def make_batch(g):
        # the 4 benchmark batches share one capacity bucket (one captured graph)
        if not pool:
            seeds = torch.randint(0, 2**31 - 1, (4 * B,), generator=g).tolist()
            ev = [lartpc_event(s, side) for s in seeds]
            if dense:
                for i in range(4):
                    chunk = ev[i * B:(i + 1) * B]
                    pool.append((torch.stack([e[0] for e in chunk]), torch.stack([e[1] for e in chunk])))
            else:
                allb = sparse_collate(ev, bucket=2048)
                for i in range(4):
                    pool.append(tuple(t[i * B:(i + 1) * B] for t in allb))
        return pool.pop(0)

    desc = (f"perceiver-io-lartpc {side}x{side}x1 fourier-bands=32 latents={args.latents}x{args.channels} "
            f"layers=3x(1+3) queries={side * side} {'dense' if dense else 'sparse'}")
    return _LArHolder(model), loss_fn, make_batch, desc, 1e-3, 1e-4


def _spawn_self(args, argv) -> int:
    """``--gpus N`` without a torchrun environment: start N ranks of this script (one per GPU,
    RCCL) and return the worst exit code.  The parent only counts devices — it never initialises
    the GPU.  With no GPU at all it is a CPU dry run over gloo; with fewer than N GPUs it fails."""
    from perceiver_io_amd.parallel.launch import gpu_count, spawn

    n = gpu_count()  # no HIP call in this process
    if 0 < n < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but only {n} GPU(s) visible", file=sys.stderr)
        return 2
    if n == 0:
        print(f"bench.py: no GPU visible: CPU dry run with {args.gpus} gloo ranks", file=sys.stderr)
    argv = list(sys.argv[1:] if argv is None else argv)
    return spawn(args.gpus, [sys.executable, os.path.abspath(__file__)] + argv)


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_self(args, argv))
    # stdout carries exactly one JSON line: everything else written to fd 1 while the run is set
    # up and timed (RCCL's version banner, library notices) goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch

    from perceiver_io_amd import ops
    from perceiver_io_amd.parallel import FlatGradReducer, dist as pdist
    from perceiver_io_amd.train.engine import StepEngine

    info = pdist.init()
    world = info.world_size
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    ops.set_backend("auto" if args.backend == "hip" else args.backend)
    torch.manual_seed(1234 + info.rank)

    lit, loss_inner, make_batch, desc, lr, wd = build(args, device)
    lit.to(device)
    model = lit.model
    lar = args.config == "lartpc"  # Adam (L2 decay) + clip 10 over the trained parameters (run.py)
    params = model.trained_parameters() if lar else [p for p in model.parameters() if p.requires_grad]
    fused = args.backend == "hip" and cuda
    if fused:
        from perceiver_io_amd.ops.optim import FusedAdam, FusedAdamW

        opt = (FusedAdam(params, lr=lr, weight_decay=wd, max_grad_norm=10.0) if lar
               else FusedAdamW(params, lr=lr, weight_decay=wd))
    else:
        opt = (torch.optim.Adam if lar else torch.optim.AdamW)(params, lr=lr, weight_decay=wd)
    sched = None if lar else torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=lr, total_steps=50000, pct_start=0.1,
                                                                 cycle_momentum=False)
    reducer = None
    # PERCEIVER_BENCH_FORCE_REDUCER=1 (one GPU, diagnostics): a 1-rank RCCL group with the reducer
    # forced on and its collectives captured in the step graph — the in-graph all-reduce / fork
    # overhead of the multi-GPU path, measured without the transfers
    force_red = world == 1 and cuda and fused and os.environ.get("PERCEIVER_BENCH_FORCE_REDUCER", "0") == "1"
    if force_red:
        import torch.distributed as tdist

        if not tdist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            tdist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
        reducer = FlatGradReducer(opt.flat, in_graph=args.overlap == "off", force=True, overlap=args.overlap == "on")
        reducer.plan(model)
    if world > 1:
        from perceiver_io_amd.ops.optim import FlatParameterSpace

        flat = opt.flat if fused else FlatParameterSpace(params, with_shadow=False, replicate=False)
        reducer = FlatGradReducer(flat, wire_dtype=torch.bfloat16 if args.allreduce_dtype == "bf16" else None,
                                  overlap=args.overlap == "on")
        reducer.plan(model)  # ready points: decoder + head, layer_n — all-reduced during the backward
        reducer.broadcast_parameters(model)

    autocast = (not fused) and args.dtype == "bf16" and cuda

    def loss_fn(batch):
        if autocast:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return loss_inner(batch)
        return loss_inner(batch)

    engine = StepEngine(loss_fn, opt, sched, reducer=reducer, device=device, graph=fused and not args.no_graph,
                        bucket_update=None if args.bucket_update == "auto" else args.bucket_update == "on")
    g = torch.Generator(device="cpu").manual_seed(99 + info.rank)

    def to_dev(b):
        return tuple(t.to(device) for t in b)

    data = [to_dev(make_batch(g)) for _ in range(4)]
    for i in range(args.warmup):
        loss = engine.step(data[i % 4], ring_view=True)
    if cuda:
        torch.cuda.synchronize()
    pdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = engine.step(data[i % 4], ring_view=True)
    if cuda:
        torch.cuda.synchronize()
    pdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = pdist.all_reduce_max(dt)
    final_loss = float(loss.float().item())
    if fused:  # a persistent-kernel spin timeout or a checked-build index error invalidates the run
        ops.check_device_errors()
    # data parallelism must leave every rank with bitwise the same parameters
    from perceiver_io_amd.parallel.reducer import params_in_sync

    sync_diff = params_in_sync(reducer.flat if reducer is not None else params) if world > 1 else 0.0
    if args.profile_steps and cuda:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(args.profile_steps):
                engine.step(data[i % 4], ring_view=True)
            torch.cuda.synchronize()
        if info.is_main:
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40), file=sys.stderr)
        if args.profile_stacks and info.is_main:
            _aten_stacks(engine, data, args.profile_steps, args.profile_stacks)
    B = args.batch
    ms = dt / args.steps * 1e3
    value = B * world * args.steps / dt
    # bar: the reference's own compute measured eagerly on one MI355X (bench/baseline_measured.json,
    # recorded in BASELINE.md); weak scaling → compare against world × per-GPU reference rate
    vs = None
    if os.path.exists(BASELINE_FILE):
        try:
            key = "mlm256" if args.config == "mlm256" else args.config
            ref = json.load(open(BASELINE_FILE)).get(f"{key}_reference_samples_per_s_per_gpu")
            vs = value / (float(ref) * world) if ref else None
        except Exception:
            vs = None
    if info.is_main:
        out = {
            "metric": CONFIGS[args.config]["metric"],
            "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(vs, 3) if vs else None,
            "dtype": ("bf16" if fused else args.dtype) if cuda else "fp32",
            "data": "synthetic (random inputs of the config's shape, random-init weights)",
            "config": {"model": desc, "global_batch": B * world, "seq_len": args.seq_len,
                       "parallelism": f"dp{world}", "backend": args.backend,
                       "graph": bool(fused and not args.no_graph), "name": args.config,
                       "dist_backend": info.backend if world > 1 else None,
                       "allreduce_in_graph": bool(reducer is not None and getattr(reducer, "in_graph", False)),
                       "allreduce_overlap": sorted(reducer.points) if reducer is not None else [],
                       "allreduce_dtype": args.allreduce_dtype if world > 1 else None,
                       "bucket_update": bool(getattr(engine, "bucket_update", False))},
            "final_loss": round(final_loss, 4),
            "dist_backend": info.backend if world > 1 else None,
            "params_in_sync": sync_diff == 0.0, "params_max_abs_diff": sync_diff,
        }
        sys.stdout.flush()
        os.dup2(json_fd, 1)
        print(json.dumps(out), flush=True)
    # captured step graphs (with their in-graph collectives) go before the communicator does
    engine = None
    if cuda:
        import gc

        gc.collect()
        torch.cuda.synchronize()
    if reducer is not None:
        reducer.close()
    pdist.shutdown()


if __name__ == "__main__":
    main()
