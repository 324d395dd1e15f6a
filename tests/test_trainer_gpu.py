"""Trainer + CLI on the GPU: fused bf16 path, hipGraph-captured steps, checkpoint round trip.

The entrypoints run with the reference's DEFAULT data behaviour: the IMDB collator pads each
batch to its longest sequence (``/root/reference/data/imdb.py:52-63``) and the loaders keep
the partial last batch (``:112-126``; pl_bolts MNIST likewise) — the step engine caches one
captured graph per (bucketed) batch shape.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(task, args, tmp_path):
    from perceiver_io_amd.cli.tasks import main

    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        return main(task, args)
    finally:
        os.chdir(old)


def test_mlm_cli_fit_gpu_graph(tmp_path):
    from perceiver_io_amd.train.checkpoint import load_checkpoint

    cli = _run("mlm", ["fit", "--data=IMDBDataModule", "--data.synthetic=true", "--data.synthetic_size=64",
                       "--data.vocab_size=500", "--data.max_seq_len=64", "--data.batch_size=8",
                       "--data.num_workers=0", "--data.pad_to_max=true", "--model.num_latents=32",
                       "--model.num_encoder_layers=2", "--model.num_encoder_self_attention_layers_per_block=2",
                       "--optimizer.lr=0.003", "--trainer.accelerator=gpu", "--trainer.devices=1",
                       "--trainer.max_steps=6", "--trainer.val_check_interval=6", "--trainer.limit_val_batches=2",
                       "--trainer.log_every_n_steps=1", "--model.masked_samples=null"], tmp_path)
    tr = cli.trainer
    assert tr.fused and tr._engine.graph_enabled and tr._engine.num_graphs == 1
    assert tr.global_step == 6
    assert type(tr.optimizers[0]).__name__ == "FusedAdamW"
    assert torch.isfinite(torch.tensor(tr.callback_metrics["train_loss"]))
    ck = [c for c in tr.callbacks if type(c).__name__ == "ModelCheckpoint"][0]
    ckpt = load_checkpoint(ck.best_model_path)
    assert ckpt["global_step"] == 6 and ckpt["optimizer_states"][0]["state"][0]["step"].item() == 6


def test_mlm_cli_default_pad_to_longest_two_epochs(tmp_path):
    """Default collator (pad to the longest sequence of each batch, lengths 8..200) and a
    partial last batch (70 = 8·8 + 6), two epochs on the graph path."""
    cli = _run("mlm", ["fit", "--data=IMDBDataModule", "--data.synthetic=true", "--data.synthetic_size=70",
                       "--data.vocab_size=500", "--data.max_seq_len=256", "--data.batch_size=8",
                       "--data.num_workers=0", "--model.num_latents=32", "--model.num_encoder_layers=2",
                       "--model.num_encoder_self_attention_layers_per_block=2", "--optimizer.lr=0.003",
                       "--trainer.accelerator=gpu", "--trainer.devices=1", "--trainer.max_epochs=2",
                       "--trainer.max_steps=18", "--trainer.limit_val_batches=2", "--trainer.log_every_n_steps=3",
                       "--model.masked_samples=null"], tmp_path)
    tr = cli.trainer
    eng = tr._engine
    assert tr.fused and eng.graph_enabled
    assert tr.global_step == 2 * 9  # ceil(70 / 8) steps per epoch, partial batch kept
    assert eng.num_graphs >= 2  # several bucketed lengths / the short last batch
    assert torch.isfinite(torch.tensor(tr.callback_metrics["train_loss"]))


def test_img_clf_cli_partial_last_batch(tmp_path):
    cli = _run("img_clf", ["fit", "--data=MNISTDataModule", "--data.synthetic=true", "--data.synthetic_size=100",
                           "--data.val_split=20", "--data.batch_size=24", "--data.num_workers=0",
                           "--model.num_latents=16", "--model.num_latent_channels=64",
                           "--model.num_encoder_layers=2", "--model.num_encoder_self_attention_layers_per_block=1",
                           "--trainer.accelerator=gpu", "--trainer.devices=1", "--trainer.max_epochs=2",
                           "--trainer.limit_val_batches=1", "--trainer.log_every_n_steps=2"], tmp_path)
    tr = cli.trainer
    n_train = 80
    steps_per_epoch = -(-n_train // 24)
    assert tr.global_step == 2 * steps_per_epoch
    assert tr._engine.graph_enabled and tr._engine.num_graphs == 1 + (n_train % 24 != 0)
    assert torch.isfinite(torch.tensor(tr.callback_metrics["train_loss"]))


def test_seq_clf_dropout_fused_under_graph(tmp_path, monkeypatch):
    """The README joint fine-tune (``--model.dropout=0.1``, ``README.md:95-107``) stays on the
    fused kernels under graph capture: the eager layer path must never run."""
    from perceiver_io_amd.models import blocks

    def boom(self, *a, **k):
        raise AssertionError("eager layer path used with dropout > 0")

    monkeypatch.setattr(blocks._FusedLayer, "eager_forward", boom)
    cli = _run("seq_clf", ["fit", "--data=IMDBDataModule", "--data.synthetic=true", "--data.synthetic_size=48",
                           "--data.vocab_size=500", "--data.max_seq_len=128", "--data.batch_size=8",
                           "--data.num_workers=0", "--model.num_latents=32", "--model.num_encoder_layers=2",
                           "--model.num_encoder_self_attention_layers_per_block=2", "--model.dropout=0.1",
                           "--optimizer.lr=0.0001", "--trainer.accelerator=gpu", "--trainer.devices=1",
                           "--trainer.max_epochs=2", "--trainer.limit_val_batches=1",
                           "--trainer.log_every_n_steps=2"], tmp_path)
    tr = cli.trainer
    assert tr.fused and tr._engine.graph_enabled and tr._engine.num_graphs >= 1
    assert tr.global_step == 2 * 6
    assert torch.isfinite(torch.tensor(tr.callback_metrics["train_loss"]))



def test_persist_spin_timeout_raises_in_trainer(tmp_path):
    """A bounded-spin timeout inside the persistent self-attention block forward (csrc/persist.hip
    ``wait_count``) must stop training, not corrupt it silently: with a test-only spin bound of
    0 polls the tiles that wait for their sample's next-layer rows give up, the kernel sets its
    sticky error word, and the Trainer's logging-step check raises naming the kernel."""
    from perceiver_io_amd.ops import ext

    K = ext.require()
    K.persist_errors(True)
    K.persist_set_spin_limit(0)
    try:
        with pytest.raises(RuntimeError, match="sa_block_fwd_kernel"):
            _run("mlm", ["fit", "--data=IMDBDataModule", "--data.synthetic=true", "--data.synthetic_size=64",
                         "--data.vocab_size=500", "--data.max_seq_len=64", "--data.batch_size=16",
                         "--data.num_workers=0", "--data.pad_to_max=true", "--model.num_latents=256",
                         "--model.num_latent_channels=64", "--model.num_encoder_self_attention_heads=4",
                         "--model.num_encoder_layers=2", "--model.num_encoder_self_attention_layers_per_block=4",
                         "--optimizer.lr=0.003", "--trainer.accelerator=gpu", "--trainer.devices=1",
                         "--trainer.max_steps=3", "--trainer.limit_val_batches=0",
                         "--trainer.log_every_n_steps=1", "--model.masked_samples=null"], tmp_path)
    finally:
        K.persist_set_spin_limit(1 << 21)
        K.persist_errors(True)
