"""Data parallelism on CPU with the gloo backend (world size 2): flat-buffer gradient
all-reduce equals single-process large-batch gradients, parameter broadcast, sharded
sampler, and a 2-rank Trainer.fit that checkpoints on rank 0 only."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _mlm(seed):
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    torch.manual_seed(seed)
    return LitMaskedLanguageModel(vocab_size=200, max_seq_len=32,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=8, num_latent_channels=32, num_encoder_layers=2,
                                  num_encoder_self_attention_layers_per_block=1)


def _worker_reduce(rank, world, port, out):
    _env(rank, world, port)
    from perceiver_io_amd.ops.optim import FlatParameterSpace
    from perceiver_io_amd.parallel import FlatGradReducer, dist

    dist.init(device_type="cpu")
    lit = _mlm(seed=rank)  # different init per rank → broadcast must fix it
    model = lit.model
    flat = FlatParameterSpace(model.parameters(), with_shadow=False)
    red = FlatGradReducer(flat, bucket_bytes=64 << 10)
    red.broadcast_parameters(model)
    g = torch.Generator().manual_seed(7)
    x = torch.randint(3, 200, (8, 32), generator=g)
    pad = torch.zeros(8, 32, dtype=torch.bool)
    xm, lab = model.masking(x, pad, generator=torch.Generator().manual_seed(11))
    # reference: full batch in this process (mean over all selected tokens of both halves)
    flat.zero_grad()
    full = model.loss(x, pad, labels=lab, x_masked=xm)
    full.backward()
    ref = flat.grad.clone()
    # DDP: each rank its half; loss normalised by the global selected count → exact sum
    flat.zero_grad()
    half = slice(rank * 4, rank * 4 + 4)
    n_loc = (lab[half] != -100).sum()
    n_tot = (lab != -100).sum()
    loss = model.loss(x[half], pad[half], labels=lab[half], x_masked=xm[half]) * (n_loc.float() / n_tot.float())
    loss.backward()
    red.finish()
    out[rank] = (flat.data.clone(), (flat.grad - ref).abs().max().item(), ref.abs().max().item(), len(red.buckets))
    dist.shutdown()


def test_flat_grad_allreduce_equals_full_batch():
    world, port = 2, _port()
    out = mp.Manager().dict()
    mp.spawn(_worker_reduce, args=(world, port, out), nprocs=world, join=True)
    p0, p1 = out[0][0], out[1][0]
    assert torch.equal(p0, p1)  # broadcast from rank 0
    for r in range(world):
        err, scale, nb = out[r][1], out[r][2], out[r][3]
        assert err < 1e-5 * max(scale, 1.0), (r, err, scale)
        assert nb >= 2  # bucketed


def test_sharded_sampler_partitions():
    from perceiver_io_amd.parallel import ShardedSampler

    n = 103
    shards = [list(ShardedSampler(n, r, 4, shuffle=True, seed=3)) for r in range(4)]
    assert all(len(s) == 26 for s in shards)
    seen = set().union(*map(set, shards))
    assert seen == set(range(n))
    s = ShardedSampler(n, 0, 4, shuffle=True, seed=3)
    a = list(s)
    s.set_epoch(1)
    assert list(s) != a


def _worker_fit(rank, world, port, tmp, out):
    _env(rank, world, port)
    os.chdir(tmp)
    from perceiver_io_amd.cli.tasks import main

    cli = main("img_clf", ["fit", "--data=MNISTDataModule", "--data.synthetic=true", "--data.synthetic_size=64",
                           "--data.batch_size=8", "--data.num_workers=0", "--data.val_split=16",
                           "--trainer.accelerator=cpu", "--trainer.max_epochs=1", "--trainer.limit_train_batches=2",
                           "--trainer.limit_val_batches=1", "--model.num_latents=8", "--model.num_latent_channels=32",
                           "--model.num_encoder_layers=1", "--model.num_encoder_self_attention_layers_per_block=1",
                           "--trainer.enable_progress_bar=false"])
    params = torch.cat([p.detach().reshape(-1) for p in cli.model.parameters()])
    ck = [c for c in cli.trainer.callbacks if type(c).__name__ == "ModelCheckpoint"][0]
    out[rank] = (params, cli.trainer.world_size, ck.best_model_path)
    from perceiver_io_amd.parallel import dist

    dist.shutdown()


def test_two_rank_trainer_fit(tmp_path):
    world, port = 2, _port()
    out = mp.Manager().dict()
    mp.spawn(_worker_fit, args=(world, port, str(tmp_path), out), nprocs=world, join=True)
    assert out[0][1] == 2 and out[1][1] == 2
    assert torch.allclose(out[0][0], out[1][0])  # replicas stay in sync
    assert os.path.exists(out[0][2])


def test_bench_self_spawns_ranks_cpu_dry_run():
    """``python bench.py --gpus 2`` without a torchrun environment starts 2 ranks itself (a CPU
    dry run over gloo here); the JSON line reports both and that their parameters agree."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "2", "--seq-len", "32", "--latents", "16", "--channels", "32", "--vocab", "300"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert [ln for ln in r.stdout.splitlines() if ln.strip()] == lines, r.stdout  # nothing else on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["dist_backend"] == "gloo" and out["params_in_sync"] is True
    assert out["config"]["allreduce_overlap"] == []  # default: one all-reduce after the backward
    assert out["config"]["bucket_update"] is False
