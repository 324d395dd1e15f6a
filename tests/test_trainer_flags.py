"""Trainer flags of scripts/trainer.yaml that the README runs leave at their defaults but a user of
the reference can turn on: gradient accumulation (`accumulate_grad_batches`,
trainer.yaml:33), gradient clipping (`gradient_clip_val`, :16-17), `terminate_on_nan` (:71),
`fast_dev_run` (:32); plus the bench.py output contract on the CPU path."""
import json
import math
import os
import subprocess
import sys

import pytest
import torch

from perceiver_io_amd.train.engine import StepEngine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _linear_pair(seed=0):
    torch.manual_seed(seed)
    a = torch.nn.Sequential(torch.nn.Linear(6, 8), torch.nn.GELU(), torch.nn.Linear(8, 3))
    b = torch.nn.Sequential(torch.nn.Linear(6, 8), torch.nn.GELU(), torch.nn.Linear(8, 3))
    b.load_state_dict(a.state_dict())
    return a, b


def test_accumulated_micro_batches_equal_one_large_batch():
    """accumulate=2 over two equal halves == one step over the concatenated batch (mean losses)."""
    a, b = _linear_pair()
    oa = torch.optim.AdamW(a.parameters(), lr=1e-2)
    ob = torch.optim.AdamW(b.parameters(), lr=1e-2)
    ce = torch.nn.CrossEntropyLoss()
    ea = StepEngine(lambda bt: ce(a(bt[0]), bt[1]), oa, accumulate=1)
    eb = StepEngine(lambda bt: ce(b(bt[0]), bt[1]), ob, accumulate=2)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        x, y = torch.randn(8, 6, generator=g), torch.randint(0, 3, (8,), generator=g)
        ea.step((x, y))
        eb.step([(x[:4], y[:4]), (x[4:], y[4:])])
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, atol=1e-6, rtol=1e-5)


def test_fused_adamw_grad_clipping_matches_clip_grad_norm():
    """FusedAdamW(max_grad_norm) == torch clip_grad_norm_ + AdamW (the eager Lightning path)."""
    from perceiver_io_amd.ops.optim import FusedAdamW

    a, b = _linear_pair(3)
    oa = torch.optim.AdamW(a.parameters(), lr=5e-2, weight_decay=0.01)
    ob = FusedAdamW(b.parameters(), lr=5e-2, weight_decay=0.01, max_grad_norm=0.05)
    g = torch.Generator().manual_seed(2)
    for _ in range(4):
        x = torch.randn(16, 6, generator=g) * 10
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
        norm = torch.nn.utils.clip_grad_norm_(a.parameters(), 0.05)
        assert norm > 0.05  # clipping is active in this test
        oa.step()
        ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, atol=1e-5, rtol=1e-4)


def _run_cli(task, tmp_path, *flags):
    from perceiver_io_amd.cli.tasks import main as cli_main

    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        return cli_main(task, list(flags))
    finally:
        os.chdir(old)


IMG_FLAGS = ["--data=MNISTDataModule", "--data.synthetic=true", "--data.synthetic_size=80", "--data.batch_size=8",
             "--data.num_workers=0", "--data.val_split=16", "--model.num_encoder_layers=1",
             "--model.num_encoder_self_attention_layers_per_block=1", "--trainer.limit_val_batches=1"]


def test_terminate_on_nan_stops_training(tmp_path, monkeypatch):
    from perceiver_io_amd.tasks import LitClassifier

    orig = LitClassifier.step

    def nan_step(self, batch):
        loss, acc = orig(self, batch)
        return loss * float("nan"), acc

    monkeypatch.setattr(LitClassifier, "step", nan_step)
    with pytest.raises(ValueError, match="non-finite"):
        _run_cli("img_clf", tmp_path, "fit", *IMG_FLAGS, "--trainer.max_epochs=1", "--trainer.limit_train_batches=4",
                 "--trainer.log_every_n_steps=1", "--trainer.terminate_on_nan=true", "--trainer.num_sanity_val_steps=0")


def test_fast_dev_run_and_accumulation_through_cli(tmp_path):
    cli = _run_cli("img_clf", tmp_path, "fit", *IMG_FLAGS, "--trainer.fast_dev_run=true")
    assert cli.trainer.global_step == 1
    cli = _run_cli("img_clf", tmp_path, "fit", *IMG_FLAGS, "--trainer.max_epochs=1", "--trainer.limit_train_batches=4",
                   "--trainer.accumulate_grad_batches=2", "--trainer.gradient_clip_val=0.5",
                   "--trainer.log_every_n_steps=1")
    assert cli.trainer.global_step == 2  # 4 micro-batches / 2 per optimizer step
    assert math.isfinite(cli.trainer.callback_metrics.get("train_loss", float("nan")))


def test_bench_json_contract_cpu():
    """bench.py prints ONE JSON line with the driver's fields (CPU, torch backend, tiny shape)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, "bench.py", "--config", "mlm256", "--backend", "torch", "--dtype", "fp32",
                          "--batch", "2", "--seq-len", "32", "--latents", "8", "--vocab", "64", "--steps", "2",
                          "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    assert [l for l in out.stdout.splitlines() if l.strip()] == lines  # nothing else on stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1 and rec["higher_is_better"] is True
    assert rec["scaling"] == "weak" and rec["value"] > 0
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(rec["config"])
    assert rec["config"]["global_batch"] == 2 and rec["config"]["seq_len"] == 32


def test_allreduce_dtype_flag(tmp_path):
    """--trainer.allreduce_dtype (the gradient all-reduce wire format, SURVEY C-03) reaches the trainer;
    a bad value is rejected.  The bf16 wire itself is exercised on 2 gloo ranks in
    test_ddp_engine.py::test_bf16_wire_format_close_to_fp32."""
    from perceiver_io_amd.train.trainer import Trainer

    cli = _run_cli("img_clf", tmp_path, "fit", *IMG_FLAGS, "--trainer.fast_dev_run=true",
                   "--trainer.allreduce_dtype=bf16")
    assert cli.trainer.allreduce_dtype == torch.bfloat16 and cli.trainer.global_step == 1
    with pytest.raises(ValueError, match="allreduce_dtype"):
        Trainer(logger=False, allreduce_dtype="fp8")


def test_gpu_count_respects_visible_devices(monkeypatch):
    """The launcher parent counts GPUs without initialising HIP (no HIP call in this process)."""
    from perceiver_io_amd.parallel.launch import gpu_count

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3,5")
    assert gpu_count() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert gpu_count() == 0


def test_topology_gpu_count_skips_unopenable_render_nodes(tmp_path):
    """A container that sees only some of the host's render nodes still lists every host GPU in
    the KFD topology: only nodes with SIMDs whose /dev/dri/renderD<minor> is openable count (the
    filter ROCr applies), so devices=-1 never starts more ranks than usable GPUs."""
    import os

    from perceiver_io_amd.parallel.launch import topology_gpu_count

    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    # node 0: the CPU (no SIMDs); nodes 1-4: GPUs with render minors 128..131
    for i, (simds, minor) in enumerate([(0, 0), (256, 128), (256, 129), (256, 130), (256, 131)]):
        d = topo / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simds}\ndrm_render_minor {minor}\n")
    for minor in (128, 130):  # only two render nodes are present and accessible here
        (dri / f"renderD{minor}").write_text("")
    assert topology_gpu_count(str(topo), str(dri)) == 2
    os.chmod(dri / "renderD130", 0o000)
    if not os.access(dri / "renderD130", os.R_OK):  # (root ignores the mode bits)
        assert topology_gpu_count(str(topo), str(dri)) == 1
    assert topology_gpu_count(str(tmp_path / "missing"), str(dri)) is None
