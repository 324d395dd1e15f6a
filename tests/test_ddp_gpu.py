"""Data parallelism on the GPU (one MI355X): the step engine's hipGraph path with the reducer.

* 2 ranks on the one card over gloo (RCCL refuses two ranks on one device): the captured
  forward/backward replays, the all-reduce + fused AdamW run after it (gloo collectives are not
  capturable).  Deterministic mode: after 5 steps both ranks hold bitwise-identical parameters,
  equal to the same ranks' eager steps.
* RCCL collectives INSIDE the step graph (the 8-GPU path, ``in_graph``), on a 1-rank RCCL group
  with the reducer forced on: the ready points fire during capture, their all-reduces run on the
  side stream inside the graph, and the replayed steps equal the plain single-GPU graph bitwise.
"""
import gc
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

# an RCCL failure (e.g. the one abort seen in round 5 inside test_rccl_collectives_inside_the_step_graph,
# which printed no reason) names its cause on stderr
os.environ.setdefault("NCCL_DEBUG", "WARN")

pytestmark = pytest.mark.gpu

STEPS = 5


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=0):
    from perceiver_io_amd import ops
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    ops.set_deterministic(True)
    ops.masking.reset_mask_state()  # recreated from the seeded generator at the first masking
    torch.manual_seed(seed)
    lit = LitMaskedLanguageModel(vocab_size=1000, max_seq_len=128,
                                 optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                 num_latents=64, num_latent_channels=64, num_encoder_layers=3,
                                 num_encoder_self_attention_layers_per_block=2, masked_samples=None)
    return lit.model.cuda()


def _data(rank, n):
    """Batches with their masking drawn up front (ids, pad, labels, masked ids): the capture
    warm-ups of the graph path run extra forwards, which would advance the device masking RNG
    and make graph and eager runs see different masks."""
    from perceiver_io_amd.models.perceiver import TextMasking

    g = torch.Generator().manual_seed(123 + rank)
    masking = TextMasking(1000)
    out = []
    for _ in range(n):
        ids = torch.randint(3, 1000, (8, 128), generator=g)
        pad = torch.zeros(8, 128, dtype=torch.bool)
        pad[2, 100:] = True
        xm, lab = masking(ids, pad, generator=g)
        out.append(tuple(t.cuda() for t in (ids, pad, lab, xm)))
    return out


def _run(model, red, graph, data):
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
    if red is not None:
        red = red(opt.flat)
        red.plan(model)
        red.broadcast_parameters(model)
    eng = StepEngine(lambda b: model.loss(b[0], b[1], labels=b[2], x_masked=b[3]), opt, reducer=red, device="cuda", graph=graph)
    for b in data:
        eng.step(b)
    torch.cuda.synchronize()
    return opt, red, eng


def _worker_gloo(rank, world, port, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PERCEIVER_DIST_BACKEND="gloo")
    from perceiver_io_amd.parallel import FlatGradReducer, dist
    from perceiver_io_amd.parallel.reducer import params_in_sync

    dist.init()
    res = {}
    for graph in (True, False):
        model = _setup()
        opt, red, eng = _run(model, lambda f: FlatGradReducer(f, overlap=True), graph, _data(rank, STEPS))
        res[graph] = dict(params=opt.flat.data.cpu(), sync=params_in_sync(opt.flat), in_graph=red.in_graph,
                          log=list(red.launch_log), replays=eng.replays)
        red.close()
    out[rank] = res
    dist.shutdown()


def test_two_ranks_graph_steps_bitwise_in_sync():
    world, port = 2, _port()
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_worker_gloo, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        g, e = out[r][True], out[r][False]
        assert g["sync"] == 0.0 and e["sync"] == 0.0
        assert not g["in_graph"]  # gloo: the collectives run after the replayed backward
        assert g["replays"] == STEPS - 2  # 2 eager warm-up steps, then captured steps
        assert g["log"] == ["decoder", "layer_n", "layer_1_sa"] * 2  # ready points fire in the eager steps only
        assert e["log"] == ["decoder", "layer_n", "layer_1_sa"] * STEPS
        assert torch.equal(g["params"], e["params"]), (g["params"] - e["params"]).abs().max()
    assert torch.equal(out[0][True]["params"], out[1][True]["params"])


def test_rccl_collectives_inside_the_step_graph():
    import torch.distributed as tdist

    from perceiver_io_amd.parallel import FlatGradReducer

    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    try:
        data = _data(0, STEPS)
        model = _setup()
        # the default data-parallel path: one all-reduce of the whole flat gradient after the
        # backward, captured on the step's own stream (no fork), then one AdamW — all in the graph
        opt, red, eng = _run(model, lambda f: FlatGradReducer(f, in_graph=True, force=True), True, data)
        assert red.enabled and red.in_graph and not red.overlap and eng.replays == STEPS - 2
        assert red.launch_log == [] and len(red.buckets) == 1
        eng = None
        gc.collect()  # the captured graphs (with their collectives) before the reducer and the group
        torch.cuda.synchronize()
        red.close()
        ref_model = _setup()
        ref_opt, _, _ = _run(ref_model, None, True, data)
        assert torch.equal(opt.flat.data, ref_opt.flat.data), (opt.flat.data - ref_opt.flat.data).abs().max()
    finally:
        from perceiver_io_amd import ops

        ops.set_deterministic(False)
        eng = None
        gc.collect()
        torch.cuda.synchronize()
        tdist.destroy_process_group()


def test_graph_gradient_accumulation_matches_eager_and_big_batch():
    """accumulate_grad_batches = 4 on the graph path (3 "micro" replays + 1 "last" replay per
    optimizer step, no eager step after the warm-up): bitwise equal to eager accumulation in
    deterministic mode, and equal to one step on the 4× batch up to the mean-of-means weighting
    (identical here: every micro-batch selects the same number of MLM targets)."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    steps, acc = 4, 4
    data = _data(0, steps * acc)
    # equal target counts per micro-batch, so the mean of the micro means is the big-batch mean
    for i, (ids, pad, lab, xm) in enumerate(data):
        lab = torch.full_like(lab, -100)
        lab[:, 5:29] = ids[:, 5:29]  # 24 targets per row: within the MLM row capacities
        data[i] = (ids, pad, lab, xm)
    res = {}
    try:
        for mode in ("graph", "eager", "big"):
            model = _setup()
            # eps ≫ |g|: the update is ~linear in the gradient, so comparing updates compares the
            # accumulated gradients (with eps = 1e-8 Adam turns round-off in near-zero gradient
            # entries into full ±lr steps)
            opt = FusedAdamW(model.parameters(), lr=1e-2, eps=1.0, weight_decay=0.0)

            def loss_fn(b):
                return model.loss(b[0], b[1], labels=b[2], x_masked=b[3])

            if mode == "big":
                eng = StepEngine(loss_fn, opt, device="cuda", graph=False)
                for s in range(steps):
                    micro = data[s * acc:(s + 1) * acc]
                    eng.step(tuple(torch.cat([m[j] for m in micro]) for j in range(4)))
            else:
                eng = StepEngine(loss_fn, opt, device="cuda", graph=mode == "graph", accumulate=acc)
                for s in range(steps):
                    eng.step(data[s * acc:(s + 1) * acc])
            torch.cuda.synchronize()
            res[mode] = (opt.flat.data.clone(), eng.replays, eng.captures)
    finally:
        ops.set_deterministic(False)
    g, e, big = res["graph"], res["eager"], res["big"]
    assert g[2] == 2 and g[1] == (steps - 2) * acc  # micro + last graphs; eager warm-up steps 1, 2
    assert torch.equal(g[0], e[0]), (g[0] - e[0]).abs().max()
    init = _setup()
    from perceiver_io_amd.ops.optim import FlatParameterSpace

    p0 = FlatParameterSpace(list(init.parameters()), with_shadow=False).data.cuda()
    rel = ((g[0] - big[0]).norm() / (big[0] - p0).norm()).item()
    assert rel < 2e-2, rel  # bf16 kernels: different row grouping, same maths


def _data_equal_targets(rank, n):
    """Like _data, with exactly 24 MLM targets per row: every rank's loss is a mean over the same
    number of targets, so the mean of the ranks' losses is the loss of the concatenated batch."""
    out = []
    for ids, pad, lab, xm in _data(rank, n):
        lab = torch.full_like(lab, -100)
        lab[:, 5:29] = ids[:, 5:29]
        out.append((ids, pad, lab, xm))
    return out


def _worker_rccl(rank, world, port, out):
    # a fresh process per rank, one GPU each: nothing touched the GPU before this point
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PERCEIVER_DIST_BACKEND="nccl")
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.parallel import FlatGradReducer, dist
    from perceiver_io_amd.parallel.reducer import params_in_sync
    from perceiver_io_amd.train.engine import StepEngine

    dist.init()
    model = _setup()
    opt = FusedAdamW(model.parameters(), lr=1e-2, eps=1.0, weight_decay=0.0)
    red = FlatGradReducer(opt.flat)  # the default: one all-reduce after the backward, inside the graph
    red.plan(model)
    red.broadcast_parameters(model)
    eng = StepEngine(lambda b: model.loss(b[0], b[1], labels=b[2], x_masked=b[3]), opt, reducer=red, device="cuda",
                     graph=True)
    for b in _data_equal_targets(rank, STEPS):
        eng.step(b)
    torch.cuda.synchronize()
    out[rank] = dict(params=opt.flat.data.cpu(), sync=params_in_sync(opt.flat), in_graph=red.in_graph,
                     replays=eng.replays, bucket=eng.bucket_update, log=list(red.launch_log))
    red.close()
    dist.shutdown()


def test_rccl_multi_gpu_ranks_graph_steps():
    """min(#GPUs, 8) RCCL ranks, one GPU each (skipped on a one-GPU box): captured steps with the
    all-reduces inside the graph where RCCL capture works, per-bucket AdamW behind each
    all-reduce; ranks bitwise in sync after 5 steps and equal (update-relative) to one process
    stepping the concatenated batch."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs")
    world, port = min(n, 8), _port()
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_worker_rccl, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        assert out[r]["sync"] == 0.0, (r, out[r]["sync"])
        assert out[r]["replays"] == STEPS - 2 and not out[r]["bucket"] and out[r]["log"] == []
        assert torch.equal(out[r]["params"], out[0]["params"])
    # one process, the concatenated batch, same deterministic kernels
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops.optim import FlatParameterSpace, FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    try:
        model = _setup()
        p0 = FlatParameterSpace(list(_setup().parameters()), with_shadow=False).data.cuda()
        opt = FusedAdamW(model.parameters(), lr=1e-2, eps=1.0, weight_decay=0.0)
        eng = StepEngine(lambda b: model.loss(b[0], b[1], labels=b[2], x_masked=b[3]), opt, device="cuda", graph=False)
        data = [_data_equal_targets(r, STEPS) for r in range(world)]
        for s in range(STEPS):
            eng.step(tuple(torch.cat([data[r][s][j] for r in range(world)]) for j in range(4)))
        torch.cuda.synchronize()
        got = out[0]["params"].cuda()
        rel = ((got - opt.flat.data).norm() / (opt.flat.data - p0).norm()).item()
        assert rel < 2e-3, rel
    finally:
        ops.set_deterministic(False)


def _worker_gloo_overlap(rank, world, port, out):
    """Default (non-deterministic) kernels, eager steps with the ready points firing DURING the
    backward and per-bucket updates on the side stream: a bucket reduced before its gradients
    are final would leave later contributions rank-local and the ranks would drift apart."""
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PERCEIVER_DIST_BACKEND="gloo")
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.parallel import FlatGradReducer, dist
    from perceiver_io_amd.parallel.reducer import params_in_sync
    from perceiver_io_amd.train.engine import StepEngine

    dist.init()
    model = _setup()
    ops.set_deterministic(False)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
    red = FlatGradReducer(opt.flat, overlap=True)
    red.plan(model)
    red.broadcast_parameters(model)
    eng = StepEngine(lambda b: model.loss(b[0], b[1], labels=b[2], x_masked=b[3]), opt, reducer=red, device="cuda",
                     graph=False)
    sync = []
    for b in _data(rank, 6):
        eng.step(b)
        sync.append(params_in_sync(opt.flat))
    out[rank] = dict(sync=sync, log=list(red.launch_log), bucket=eng.bucket_update)
    red.close()
    dist.shutdown()


def test_two_ranks_overlapped_nondeterministic_in_sync():
    world, port = 2, _port()
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_worker_gloo_overlap, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        assert out[r]["bucket"]
        assert out[r]["log"] == ["decoder", "layer_n", "layer_1_sa"] * 6
        assert out[r]["sync"] == [0.0] * 6, out[r]["sync"]


def _worker_probe_failure(rank, port, out):
    # a fresh process: a 1-rank RCCL group whose all-reduce raises while a capture is open
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      PERCEIVER_DIST_BACKEND="nccl")
    os.environ.pop("PERCEIVER_GRAPH_COLLECTIVES", None)
    from perceiver_io_amd.ops.optim import FlatParameterSpace
    import torch.distributed as tdist

    from perceiver_io_amd.parallel import FlatGradReducer
    from perceiver_io_amd.parallel import dist as pdist

    # a real 1-rank RCCL group (dist.init() leaves a single process without one)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    pdist._INFO = pdist.DistInfo(rank=0, local_rank=0, world_size=1, backend="nccl")
    real = pdist.dist.all_reduce

    def failing(t, *a, **k):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("injected: collective not capturable")
        return real(t, *a, **k)

    pdist.dist.all_reduce = failing
    try:
        ok = pdist.graph_collectives_ok(torch.device("cuda:0"))
    finally:
        pdist.dist.all_reduce = real
    res = dict(ok=ok, capturing=torch.cuda.is_current_stream_capturing())
    # every stream still usable: a collective and a kernel on a fresh side stream, then a sync
    side = torch.cuda.Stream()
    t = torch.ones(32, device="cuda")
    with torch.cuda.stream(side):
        res["side_capturing"] = torch.cuda.is_current_stream_capturing()
        real(t)
        t.mul_(3.0)
    torch.cuda.synchronize()
    res["value"] = float(t[0])
    flat = FlatParameterSpace([torch.nn.Parameter(torch.ones(16, device="cuda"))], with_shadow=False)
    red = FlatGradReducer(flat, force=True)  # asks the (cached) probe
    res["in_graph"] = red.in_graph
    red.close()
    out[0] = res
    tdist.destroy_process_group()


def test_graph_collectives_probe_capture_failure_fails_closed():
    """The capture probe's failure branch (dist.graph_collectives_ok): a collective that raises
    inside the capture leaves no open capture behind, the probe answers False, later work on any
    stream runs, and a reducer then keeps its collectives outside the graph (in_graph False)."""
    port = _port()
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_worker_probe_failure, args=(port, out), nprocs=1, join=True)
    r = out[0]
    assert r["ok"] is False and r["in_graph"] is False
    assert not r["capturing"] and not r["side_capturing"]
    assert r["value"] == 3.0  # 1-rank all-reduce (x1) then x3


def test_rccl_overlap_and_bucket_update_variants_bitwise():
    """The data-parallel step's variants on a 1-rank RCCL group with the reducer forced on,
    deterministic kernels: ready-point all-reduces on a side stream (overlap on: collectives
    outside the step graph, after each replay) or one all-reduce inline after the backward inside
    the graph (overlap off), AdamW per bucket behind each all-reduce or one pass after all of them
    (bucket_update on / off) — the final parameters agree bit for bit (the slab reductions a
    ready point flushes run on the side stream only when every destination lies inside the
    bucket; in deterministic mode all of them stay on the compute stream)."""
    import torch.distributed as tdist

    from perceiver_io_amd import ops
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.parallel import FlatGradReducer
    from perceiver_io_amd.train.engine import StepEngine

    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    try:
        data = _data(0, STEPS)
        res = {}
        for overlap in (True, False):
            for bucket in (True, False):
                model = _setup()
                opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
                red = FlatGradReducer(opt.flat, in_graph=not overlap, force=True, overlap=overlap)
                red.plan(model)
                eng = StepEngine(lambda b, m=model: m.loss(b[0], b[1], labels=b[2], x_masked=b[3]), opt, reducer=red,
                                 device="cuda", graph=True, bucket_update=bucket)
                for b in data:
                    eng.step(b)
                torch.cuda.synchronize()
                assert eng.bucket_update == bucket and red.overlap == overlap
                res[(overlap, bucket)] = opt.flat.data.clone()
                eng = None
                import gc

                gc.collect()  # the captured graphs (with their collectives) before the reducer
                torch.cuda.synchronize()
                red.close()
        ref = res[(True, True)]
        for k, v in res.items():
            assert torch.equal(v, ref), (k, (v - ref).abs().max().item())
    finally:
        ops.set_deterministic(False)
        tdist.destroy_process_group()
