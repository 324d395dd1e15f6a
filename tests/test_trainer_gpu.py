"""Trainer + CLI on the GPU: fused bf16 path, hipGraph-captured steps, checkpoint round trip."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_mlm_cli_fit_gpu_graph(tmp_path):
    from perceiver_io_amd.cli.tasks import main
    from perceiver_io_amd.train.checkpoint import load_checkpoint

    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        cli = main("mlm", ["fit", "--data=IMDBDataModule", "--data.synthetic=true", "--data.synthetic_size=64",
                           "--data.vocab_size=500", "--data.max_seq_len=64", "--data.batch_size=8",
                           "--data.num_workers=0", "--data.pad_to_max=true", "--model.num_latents=32",
                           "--model.num_encoder_layers=2", "--model.num_encoder_self_attention_layers_per_block=2",
                           "--optimizer.lr=0.003", "--trainer.accelerator=gpu", "--trainer.devices=1",
                           "--trainer.max_steps=6", "--trainer.val_check_interval=6", "--trainer.limit_val_batches=2",
                           "--trainer.log_every_n_steps=1", "--model.masked_samples=null"])
    finally:
        os.chdir(old)
    tr = cli.trainer
    assert tr.fused and tr._engine.graph_enabled and tr._engine._graph is not None
    assert tr.global_step == 6
    assert type(tr.optimizers[0]).__name__ == "FusedAdamW"
    assert torch.isfinite(torch.tensor(tr.callback_metrics["train_loss"]))
    ck = [c for c in tr.callbacks if type(c).__name__ == "ModelCheckpoint"][0]
    ckpt = load_checkpoint(ck.best_model_path)
    assert ckpt["global_step"] == 6 and ckpt["optimizer_states"][0]["state"][0]["step"].item() == 6
