"""Task modules: masked language model, text classifier, image classifier.

Reference parity (``perceiver/lightning.py``):
  * ``LitModel``               — ``:29-55``: shared architecture hparams + defaults,
    ``save_hyperparameters``, optimizer / per-step scheduler from ``{class_path, init_args}``.
  * ``LitClassifier``          — ``:58-85``: CE loss + argmax accuracy; logs ``train_loss``,
    ``train_acc``, ``val_loss``, ``val_acc``, ``test_loss``, ``test_acc``.
  * ``LitImageClassifier``     — ``:88-126``.
  * ``LitTextClassifier``      — ``:129-171``: encoder shared with the MLM, transfer from
    ``mlm_ckpt`` (encoder) or ``clf_ckpt`` (whole model), ``freeze_encoder``.  Defect D3
    fixed (``PerceiverIO.encoder`` exists); D8: a stale nested ``mlm_ckpt`` path inside a
    ``clf_ckpt``'s hparams is skipped with a warning instead of crashing.
  * ``LitMaskedLanguageModel`` — ``:174-256``: defect D1 fixed (``TextMasking`` built from
    the tokenizer constants), sample predictions after each validation epoch.

Training loss of the MLM uses ``PerceiverMLM.loss`` (identical value, vocab head only on
selected positions); ``step`` on the ``reference`` backend reproduces the full-logits path.
"""
from __future__ import annotations

import os
import warnings
from typing import Any, List, Optional, Tuple

import torch
import torch.nn as nn

from .models import (ClassificationOutputAdapter, ImageInputAdapter, PerceiverDecoder, PerceiverEncoder, PerceiverIO,
                     PerceiverMLM, TextInputAdapter, TextMasking, TextOutputAdapter)
from .train.module import LitModuleBase, instantiate_class
from .utils.misc import freeze, predict_masked_samples
from .utils.tokenizer import MASK_TOKEN_ID, PAD_TOKEN_ID, SPECIAL_TOKENS, UNK_TOKEN_ID

# text batches are padded to a multiple of this many tokens before a graph-captured step
LENGTH_BUCKET = 64


def bucket_text_batch(batch, max_seq_len: int, multiple: int = LENGTH_BUCKET):
    """``(labels, ids, pad_mask)`` padded along the sequence to ``round_up(L, multiple)``
    (capped at ``max_seq_len``) with PAD ids and ``True`` (= padding) mask entries.

    The reference collator pads each batch to its longest sequence (``data/imdb.py:52-63``), so
    an epoch sees hundreds of lengths; captured step graphs are cached per shape, and this
    bounds the distinct shapes to ``max_seq_len / multiple``.  Semantics are unchanged: padded
    keys are masked out of every cross-attention (K-08), masking never selects PAD positions,
    and the MLM loss / classifier read no padded position."""
    y, x, m = batch
    L = x.shape[1]
    Lp = min(-(-L // multiple) * multiple, max(L, int(max_seq_len)))
    if Lp == L:
        return batch
    if m is None:
        m = torch.zeros(x.shape, dtype=torch.bool, device=x.device)
    x = torch.nn.functional.pad(x, (0, Lp - L), value=PAD_TOKEN_ID)
    m = torch.nn.functional.pad(m, (0, Lp - L), value=True)
    return y, x, m


class LitModel(LitModuleBase):
    def __init__(self,
                 optimizer_init: dict,
                 scheduler_init: Optional[dict] = None,
                 num_latents: int = 64,
                 num_latent_channels: int = 64,
                 num_encoder_layers: int = 3,
                 num_encoder_cross_attention_heads: int = 4,
                 num_encoder_self_attention_heads: int = 4,
                 num_encoder_self_attention_layers_per_block: int = 6,
                 num_decoder_cross_attention_heads: int = 4,
                 dropout: float = 0.0):
        super().__init__()
        self.save_hyperparameters()

    @property
    def latent_shape(self) -> Tuple[int, int]:
        return self.hparams.num_latents, self.hparams.num_latent_channels

    def configure_optimizers(self):
        optimizer = instantiate_class(self.parameters(), self.hparams.optimizer_init)
        if self.hparams.get("scheduler_init") is None:
            return optimizer
        scheduler = instantiate_class(optimizer, self.hparams.scheduler_init)
        return {"optimizer": optimizer,
                "lr_scheduler": {"scheduler": scheduler, "interval": "step", "frequency": 1}}


class Accuracy:
    """argmax accuracy (torchmetrics ``Accuracy`` as used at ``lightning.py:62,68``)."""

    def __call__(self, y_pred: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        return (y_pred == y).float().mean()


class LitClassifier(LitModel):
    def __init__(self, *args: Any, **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.loss = nn.CrossEntropyLoss()
        self.acc = Accuracy()

    def step(self, batch):
        logits, y = self(batch)
        loss = self.loss(logits.float(), y)
        acc = self.acc(logits.argmax(dim=-1), y)
        return loss, acc

    def training_step(self, batch, batch_idx):
        loss, acc = self.step(batch)
        self.log("train_loss", loss)
        self.log("train_acc", acc, prog_bar=True)
        return loss

    def validation_step(self, batch, batch_idx):
        loss, acc = self.step(batch)
        self.log("val_loss", loss, prog_bar=True)
        self.log("val_acc", acc, prog_bar=True)

    def test_step(self, batch, batch_idx):
        loss, acc = self.step(batch)
        self.log("test_loss", loss)
        self.log("test_acc", acc)


class LitImageClassifier(LitClassifier):
    def __init__(self, image_shape: Tuple[int, int, int], num_classes: int, *args: Any, num_frequency_bands: int = 32,
                 **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.model = self.create_model()

    def create_model(self):
        hp = self.hparams
        input_adapter = ImageInputAdapter(image_shape=tuple(hp.image_shape), num_frequency_bands=hp.num_frequency_bands)
        output_adapter = ClassificationOutputAdapter(num_classes=hp.num_classes, num_output_channels=hp.num_latent_channels)
        encoder = PerceiverEncoder(
            input_adapter=input_adapter, latent_shape=self.latent_shape, num_layers=hp.num_encoder_layers,
            num_cross_attention_heads=hp.num_encoder_cross_attention_heads,
            num_self_attention_heads=hp.num_encoder_self_attention_heads,
            num_self_attention_layers_per_block=hp.num_encoder_self_attention_layers_per_block, dropout=hp.dropout)
        decoder = PerceiverDecoder(output_adapter=output_adapter, latent_shape=self.latent_shape,
                                   num_cross_attention_heads=hp.num_decoder_cross_attention_heads, dropout=hp.dropout)
        return PerceiverIO(encoder, decoder)

    def forward(self, batch):
        x, y = batch
        return self.model(x), y


class LitTextClassifier(LitClassifier):
    def __init__(self, num_classes: int, vocab_size: int, max_seq_len: int, *args: Any, freeze_encoder: bool = False,
                 mlm_ckpt: Optional[str] = None, clf_ckpt: Optional[str] = None, **kwargs: Any):
        super().__init__(*args, **kwargs)
        encoder = LitMaskedLanguageModel.create_encoder(self.hparams, self.latent_shape)
        self.model = self.create_model(encoder)
        if mlm_ckpt is not None:
            lit = LitMaskedLanguageModel.load_from_checkpoint(mlm_ckpt)
            self.model.encoder.load_state_dict(lit.model.encoder.state_dict())
        elif clf_ckpt is not None:
            lit = LitTextClassifier.load_from_checkpoint(clf_ckpt, **_stale_ckpt_overrides(clf_ckpt))
            self.model.load_state_dict(lit.model.state_dict())
        if freeze_encoder:
            freeze(self.model.encoder)

    def create_model(self, encoder):
        hp = self.hparams
        output_adapter = ClassificationOutputAdapter(num_classes=hp.num_classes, num_output_channels=hp.num_latent_channels)
        decoder = PerceiverDecoder(output_adapter=output_adapter, latent_shape=self.latent_shape,
                                   num_cross_attention_heads=hp.num_decoder_cross_attention_heads, dropout=hp.dropout)
        return PerceiverIO(encoder, decoder)

    def forward(self, batch):
        y, x, x_mask = batch
        return self.model(x, x_mask), y

    def graph_batch(self, batch):
        return bucket_text_batch(batch, self.hparams.max_seq_len)


def _stale_ckpt_overrides(clf_ckpt: str) -> dict:
    """D8: the clf checkpoint's hparams may carry an mlm_ckpt path that no longer exists."""
    from .train.checkpoint import load_checkpoint

    hp = load_checkpoint(clf_ckpt, map_location="cpu").get("hyper_parameters", {})
    nested = hp.get("mlm_ckpt")
    if nested and not os.path.exists(nested):
        warnings.warn(f"clf_ckpt refers to missing mlm_ckpt {nested!r}; skipping the nested encoder load")
        return {"mlm_ckpt": None}
    return {}


class LitMaskedLanguageModel(LitModel):
    def __init__(self, vocab_size: int, max_seq_len: int, *args: Any, masked_samples: Optional[List[str]] = None,
                 num_predictions: int = 3, **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.model = self.create_model()
        self.loss = nn.CrossEntropyLoss()

    @staticmethod
    def create_encoder(hparams, latent_shape):
        input_adapter = TextInputAdapter(vocab_size=hparams.vocab_size, max_seq_len=hparams.max_seq_len,
                                         num_input_channels=hparams.num_latent_channels)
        return PerceiverEncoder(
            input_adapter=input_adapter, latent_shape=latent_shape, num_layers=hparams.num_encoder_layers,
            num_cross_attention_heads=hparams.num_encoder_cross_attention_heads,
            num_self_attention_heads=hparams.num_encoder_self_attention_heads,
            num_self_attention_layers_per_block=hparams.num_encoder_self_attention_layers_per_block,
            dropout=hparams.dropout)

    def create_model(self):
        hp = self.hparams
        encoder = self.create_encoder(hp, self.latent_shape)
        output_adapter = TextOutputAdapter(vocab_size=hp.vocab_size, max_seq_len=hp.max_seq_len,
                                           num_output_channels=hp.num_latent_channels)
        decoder = PerceiverDecoder(output_adapter=output_adapter, latent_shape=self.latent_shape,
                                   num_cross_attention_heads=hp.num_decoder_cross_attention_heads, dropout=hp.dropout)
        masking = TextMasking(hp.vocab_size, unk_token_id=UNK_TOKEN_ID, mask_token_id=MASK_TOKEN_ID,
                              num_special_tokens=len(SPECIAL_TOKENS))
        return PerceiverMLM(encoder, decoder, masking)

    def forward(self, batch):
        _, x, x_mask = batch
        return self.model(x, x_mask)

    def step(self, batch):
        _, x, x_mask = batch
        return self.model.loss(x, x_mask)

    def graph_batch(self, batch):
        return bucket_text_batch(batch, self.hparams.max_seq_len)

    def training_step(self, batch, batch_idx):
        loss = self.step(batch)
        self.log("train_loss", loss)
        return loss

    def validation_step(self, batch, batch_idx):
        self.log("val_loss", self.step(batch), prog_bar=True)

    def test_step(self, batch, batch_idx):
        self.log("test_loss", self.step(batch))

    def on_validation_epoch_end(self) -> None:
        if not self.hparams.get("masked_samples"):
            return
        trainer = self.trainer
        dm = getattr(trainer, "datamodule", None) if trainer is not None else None
        if dm is None or getattr(dm, "collator", None) is None:
            return
        samples = [s.replace("<MASK>", "[MASK]") for s in self.hparams.masked_samples]
        preds = predict_masked_samples(masked_samples=samples, encode_fn=dm.collator.encode, tokenizer=dm.tokenizer,
                                       model=self.model, device=self.device,
                                       num_predictions=self.hparams.num_predictions)
        text = "\n\n".join(["  \n".join([s] + ps) for s, ps in zip(samples, preds)])
        if self.logger is not None:
            self.logger.add_text("sample predictions", text, trainer.global_step)
