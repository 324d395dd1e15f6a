"""Data-parallel training through the step engine's capture/replay sequence (CPU, gloo).

The engine runs with ``graph_impl="closure"`` (``train/engine.py`` ``ClosureGraph``): the exact
sequence of the hipGraph path — eager warm-up steps, capture warm-ups with the reducer disarmed,
the captured step (ready points armed only when the collectives are in the graph), replays —
executes on CPU ranks with the fused executor's kernel emulation.  Pinned here:

* every rank ends every step with bitwise-identical parameters (the round-2 defect: the
  decoder bucket dropped from every captured step, ``VERDICT.md`` What's weak #1);
* the graph path equals the eager path bitwise, for the collectives inside the graph
  (``in_graph=True``, RCCL) and after it (``in_graph=False``, gloo);
* overlapped ready points (``decoder``, ``layer_n``) give the same bits as no overlap;
* gradient accumulation (2 micro-batches, micro + last graphs) equals eager accumulation
  bitwise and a single process over all ranks' micro-batches within fp32 round-off;
* the reducer protocol fails loudly on a stale launch.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

V, L = 200, 32


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _fused_on_cpu():
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import emulation, ext

    ext._mod = emulation
    ops.use_hip = lambda t: True


def _model():
    """64 × 64 latents, 4 heads: the headline's fused path (one-launch self-attention layers, the
    layer_n query projection computed by layer_1's last kernel and its backward handed back)."""
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    torch.manual_seed(0)
    return LitMaskedLanguageModel(vocab_size=V, max_seq_len=L,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=64, num_latent_channels=64, num_encoder_layers=3,
                                  num_encoder_self_attention_layers_per_block=2).model


def _batches(rank, steps, acc):
    """Per rank, per step: ``acc`` micro-batches (x, pad, labels, masked x) with fixed masking."""
    model = _model()
    out = []
    for s in range(steps):
        micro = []
        for m in range(acc):
            g = torch.Generator().manual_seed(1000 * rank + 10 * s + m)
            x = torch.randint(3, V, (3, L), generator=g)
            pad = torch.zeros(3, L, dtype=torch.bool)
            pad[1, 20 + m:] = True
            xm, lab = model.masking(x, pad, generator=torch.Generator().manual_seed(77 + 1000 * rank + 10 * s + m))
            micro.append((x, pad, lab, xm))
        out.append(micro)
    return out


def _loss_fn(model):
    def f(b):
        x, pad, lab, xm = b
        return model.loss(x, pad, labels=lab, x_masked=xm)
    return f


def _worker(rank, world, port, cases, steps, out):
    _env(rank, world, port)
    _fused_on_cpu()
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.parallel import FlatGradReducer, dist
    from perceiver_io_amd.parallel.reducer import params_in_sync
    from perceiver_io_amd.train.engine import StepEngine

    dist.init(device_type="cpu")
    res = {}
    for name, (graph, in_graph, overlap, acc, *extra) in cases.items():
        bucket = extra[0] if extra else True
        wire = extra[1] if len(extra) > 1 else None
        model = _model()
        opt = FusedAdamW(model.parameters(), lr=1e-2, eps=0.1, weight_decay=0.01)
        red = FlatGradReducer(opt.flat, bucket_bytes=None if overlap is None else 16 << 10, overlap=overlap,
                              in_graph=in_graph, wire_dtype=wire)
        red.plan(model)
        red.broadcast_parameters(model)
        eng = StepEngine(_loss_fn(model), opt, reducer=red, graph=graph, accumulate=acc, warmup_eager=1,
                         graph_impl="closure" if graph else None, bucket_update=bucket)
        data = _batches(rank, steps, acc)
        sync = []
        for s in range(steps):
            eng.step(data[s] if acc > 1 else data[s][0])
            sync.append(params_in_sync(opt.flat))
        res[name] = dict(params=opt.flat.data.clone(), sync=sync, log=list(red.launch_log), points=dict(red.points),
                         replays=eng.replays, captures=eng.captures, buckets=list(red.buckets),
                         bucket_mode=eng.bucket_update)
        red.close()
    out[rank] = res
    dist.shutdown()


CASES = {
    # name: (graph, in_graph, overlap, accumulate[, per-bucket optimizer updates (default on)[, wire dtype]])
    "eager": (False, False, True, 1),
    "eager_nooverlap": (False, False, False, 1),
    "graph_in": (True, True, True, 1),
    "graph_out": (True, False, True, 1),
    "eager_acc2": (False, False, True, 2),
    "graph_in_acc2": (True, True, True, 2),
    "graph_out_acc2": (True, False, True, 2),
    # one whole-buffer AdamW after finish() (the pre-bucket-update path)
    "eager_whole": (False, False, True, 1, False),
    "graph_in_whole": (True, True, True, 1, False),
    "graph_out_whole": (True, False, True, 1, False),
    "graph_in_acc2_whole": (True, True, True, 2, False),
    # bf16 on the wire (SURVEY C-03's optional format)
    "eager_bf16wire": (False, False, True, 1, True, torch.bfloat16),
    # the defaults (overlap=None, bucket_update=None): one all-reduce of the whole buffer after the
    # backward, one AdamW pass — in and out of the graph
    "eager_default": (False, False, None, 1, None),
    "graph_in_default": (True, True, None, 1, None),
}
STEPS = 4


@pytest.fixture(scope="module")
def ddp_runs():
    world, port = 2, _port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, CASES, STEPS, out), nprocs=world, join=True)
    return {r: dict(out[r]) for r in range(world)}, world


def test_ranks_bitwise_in_sync_every_step(ddp_runs):
    runs, world = ddp_runs
    for name in CASES:
        for r in range(world):
            assert runs[r][name]["sync"] == [0.0] * STEPS, (name, r, runs[r][name]["sync"])
        assert torch.equal(runs[0][name]["params"], runs[1][name]["params"]), name


def test_graph_path_equals_eager_bitwise(ddp_runs):
    runs, _ = ddp_runs
    p = {n: runs[0][n]["params"] for n in CASES}
    assert torch.equal(p["eager"], p["eager_nooverlap"])  # ready points do not change the bits
    assert torch.equal(p["eager"], p["graph_in"])
    assert torch.equal(p["eager"], p["graph_out"])
    assert torch.equal(p["eager_acc2"], p["graph_in_acc2"])
    assert torch.equal(p["eager_acc2"], p["graph_out_acc2"])
    assert not torch.equal(p["eager"], p["eager_acc2"])
    assert torch.equal(p["eager"], p["eager_default"])
    assert torch.equal(p["eager"], p["graph_in_default"])


def test_default_is_one_inline_allreduce(ddp_runs):
    """The default data-parallel step: no ready points, the whole flat gradient as one bucket,
    one optimizer pass (profiles/r6_reducer_ab.md: the side-stream overlap costs more than it
    hides at these gradient sizes)."""
    runs, _ = ddp_runs
    for name in ("eager_default", "graph_in_default"):
        r = runs[0][name]
        assert r["log"] == [] and r["points"] == {} and not r["bucket_mode"], name
        assert len(r["buckets"]) == 1 and r["buckets"][0][0] == 0, (name, r["buckets"])


def test_bucket_updates_equal_whole_buffer_update_bitwise(ddp_runs):
    """AdamW run per bucket right behind each all-reduce (overlapping the backward) gives exactly
    the bits of one whole-buffer update after finish(), on every path."""
    runs, _ = ddp_runs
    r = runs[0]
    assert r["eager"]["bucket_mode"] and not r["eager_whole"]["bucket_mode"]
    for a, b in (("eager", "eager_whole"), ("graph_in", "graph_in_whole"), ("graph_out", "graph_out_whole"),
                 ("graph_in_acc2", "graph_in_acc2_whole")):
        assert torch.equal(r[a]["params"], r[b]["params"]), (a, b)


def test_bf16_wire_format_close_to_fp32(ddp_runs):
    """bf16 all-reduce (half the bytes on xGMI): ranks stay bitwise in sync (checked for every
    case above) and the trajectory stays within bf16 rounding of the fp32-wire one."""
    runs, _ = ddp_runs
    a, b = runs[0]["eager_bf16wire"]["params"], runs[0]["eager"]["params"]
    init = _flat_init()
    rel = ((a - b).norm() / (b - init).norm()).item()
    assert 0.0 < rel < 5e-2, rel


def _flat_init():
    from perceiver_io_amd.ops.optim import FlatParameterSpace

    return FlatParameterSpace(list(_model().parameters()), with_shadow=False).data


def test_ready_points_fire_where_expected(ddp_runs):
    runs, _ = ddp_runs
    r = runs[0]
    order = ["decoder", "layer_n", "layer_1_sa"]
    assert set(r["eager"]["points"]) == set(order)
    # backward order: the decoder first, then layer_n, then layer_1's self-attention block — once
    # per optimizer step
    assert r["eager"]["log"] == order * STEPS
    assert r["eager_nooverlap"]["log"] == []
    # collectives in the graph: every replay's backward launches them (closure replays run Python);
    # not capturable: only the eager warm-up step does, the replays reduce everything in finish()
    assert r["graph_in"]["log"] == order * STEPS
    assert r["graph_out"]["log"] == order
    # accumulation: ready points only in the last micro-batch's backward
    assert r["eager_acc2"]["log"] == order * STEPS
    assert r["graph_in_acc2"]["log"] == order * STEPS
    assert r["graph_in_acc2"]["captures"] == 2 and r["graph_in_acc2"]["replays"] == 2 * (STEPS - 1)
    # disjoint buckets covering the whole flat buffer
    bk = sorted(r["eager"]["buckets"])
    assert bk[0][0] == 0 and all(a[1] == b[0] for a, b in zip(bk, bk[1:]))


def test_accumulation_matches_single_process(monkeypatch):
    """Single process, plain torch AdamW over the mean of all ranks' micro-batch losses (the DDP +
    accumulate gradient), against the 2-rank graph-accumulated run."""
    world, port = 2, _port()
    out = mp.Manager().dict()
    cases = {"graph_in_acc2": CASES["graph_in_acc2"]}
    mp.spawn(_worker, args=(world, port, cases, 3, out), nprocs=world, join=True)
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import emulation, ext

    monkeypatch.setattr(ext, "_mod", emulation)  # the fused executor on CPU, for this test only
    monkeypatch.setattr(ops, "use_hip", lambda t: True)
    model = _model()
    params = list(model.parameters())
    opt = torch.optim.AdamW(params, lr=1e-2, eps=0.1, weight_decay=0.01)
    data = {r: _batches(r, 3, 2) for r in range(world)}
    f = _loss_fn(model)
    for s in range(3):
        opt.zero_grad()
        loss = sum(f(b) for r in range(world) for b in data[r][s]) / (2 * world)
        loss.backward()
        opt.step()
    from perceiver_io_amd.ops.optim import FlatParameterSpace

    ref = FlatParameterSpace(params, with_shadow=False).data
    got = out[0]["graph_in_acc2"]["params"]
    init = FlatParameterSpace(list(_model().parameters()), with_shadow=False).data
    # the emulation rounds activations to bf16 like the kernels: after the first update the two
    # runs' weights differ by fp32 round-off, which flips a few bf16 roundings, so compare the
    # parameter UPDATES — a missing or rank-local bucket would be off by O(1) of them
    d_got, d_ref = got - init, ref - init
    rel = ((d_got - d_ref).norm() / d_ref.norm()).item()
    assert rel < 2e-3, rel


def _worker_protocol(rank, world, port, out):
    _env(rank, world, port)
    _fused_on_cpu()
    from perceiver_io_amd.ops.optim import FlatParameterSpace
    from perceiver_io_amd.parallel import FlatGradReducer, dist

    dist.init(device_type="cpu")
    model = _model()
    flat = FlatParameterSpace(model.parameters(), with_shadow=False, replicate=False)
    red = FlatGradReducer(flat, bucket_bytes=16 << 10, overlap=True)
    red.plan(model)
    f = _loss_fn(model)
    b = _batches(rank, 1, 1)[0][0]
    res = {}
    # a backward while disarmed (capture warm-ups) launches nothing and leaves no state behind
    f(b).backward()
    res["disarmed_launches"] = red.early_launches
    flat.zero_grad()
    red.arm()
    f(b).backward()
    res["armed_launches"] = red.early_launches
    try:
        red.arm()  # the previous backward's buckets were never finished
        res["stale"] = "no error"
    except RuntimeError as e:
        res["stale"] = str(e)
    red.finish()
    red.arm()
    red.finish()  # armed but no backward: everything reduced in finish(), once
    red.close()
    out[rank] = res
    dist.shutdown()


def test_reducer_protocol_fails_loudly_on_stale_launch():
    world, port = 2, _port()
    out = mp.Manager().dict()
    mp.spawn(_worker_protocol, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        assert out[r]["disarmed_launches"] == 0
        assert out[r]["armed_launches"] == 3  # decoder, layer_n, layer_1_sa
        assert "never finished" in out[r]["stale"]
