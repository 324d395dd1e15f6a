"""LArTPC per-pixel segmentation model (reference ``run.py:72-124``) and its sparse
execution.

The reference runs Perceiver IO densely on a 512×512 wire-plane image: 262,144 keys through the
encoder cross-attention (K/V LayerNorm + projection for every pixel), with the zero pixels
masked as keys (``mask = x == 0``, ``run.py:117``), and 262,144 output queries per sample
through the decoder, followed by a class-weighted cross-entropy whose background weight is 0
(``run.py:238-241``).  About 1–3 % of the pixels are non-zero, so nearly all of that work is
discarded.

``LArPerceiver.sparse_loss`` computes the same loss and gradients from the pixels that matter:

* **encoder**: masked keys get exactly zero attention weight, so the encoder output depends
  only on the non-zero pixels.  Their ``[pixel ‖ Fourier PE]`` rows are gathered (the PE by flat
  pixel index, ``sparse_inputs``) and the encoder runs over those keys alone,
  with the padding of the per-batch capacity masked.
* **decoder**: a pixel whose class weight is 0 contributes nothing to the loss, so its output
  query receives a zero gradient.  Only the queries of weighted pixels are decoded
  (``PerceiverDecoder.hidden_at``), and the cross-entropy is the weighted mean over them.

Parameter gradients (including the zero rows of the 262,144 × C output-query table) equal the
dense computation's.  ``tests/test_lartpc.py`` checks this against the dense eager model.
``forward`` keeps the dense per-pixel logits for inference.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch
import torch.nn.functional as F

from .adapters import ClassificationOutputAdapter, ImageInputAdapter
from .perceiver import PerceiverDecoder, PerceiverEncoder, PerceiverIO
from .uresnet import UResNet

NUM_CLASSES = 3
CLASS_WEIGHTS = (0.0, 1.0, 1.0)  # background, track, shower (reference run.py:238-240)


def sparse_inputs(adapter: ImageInputAdapter, values: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """``[pixel channels ‖ Fourier PE]`` rows at flat pixel positions ``index`` (B, K):
    ``values`` (B, K, C_img) → (B, K, Kin), the rows ``adapter(x)`` has at those positions."""
    pe = adapter.position_encoding
    b, k = index.shape
    rows = pe.index_select(0, index.reshape(-1)).view(b, k, pe.shape[1])
    return torch.cat([values.to(pe.dtype).view(b, k, -1), rows], dim=-1)


class LArPerceiver(torch.nn.Module):
    """The reference ``LAr_Perceiver`` (``run.py:72-124``): Fourier-encoded 512×512×1 input,
    32×64 latents, 3 × (1 cross + 3 self-attention) layers with 4 heads, a 1-head decoder with
    one output query per pixel and a 3-way classifier.  The U-ResNet is built alongside, unused in
    ``forward``, as in the reference (its parameters stay in the state dict)."""

    def __init__(self, size: int = 512, latents: Tuple[int, int] = (32, 64), bands: int = 32):
        super().__init__()
        n, c = latents
        enc = PerceiverEncoder(ImageInputAdapter((size, size, 1), bands), (n, c), num_layers=3,
                               num_cross_attention_heads=4, num_self_attention_heads=4,
                               num_self_attention_layers_per_block=3, dropout=0.0)
        dec = PerceiverDecoder(ClassificationOutputAdapter(num_classes=NUM_CLASSES, num_outputs=size * size,
                                                           num_output_channels=c),
                               (n, c), num_cross_attention_heads=1, dropout=0.0)
        self.size = size
        self.perceiver = PerceiverIO(enc, dec)
        self.uresnet = UResNet(num_classes=NUM_CLASSES, input_channels=c, inplanes=16)

    @property
    def encoder(self) -> PerceiverEncoder:
        return self.perceiver.encoder

    @property
    def decoder(self) -> PerceiverDecoder:
        return self.perceiver.decoder

    def trained_parameters(self):
        """The parameters that receive gradients (the unused U-ResNet excluded)."""
        return list(self.perceiver.parameters())

    def forward(self, img):
        """Dense per-pixel logits ``(B, 3, H·W)`` (the reference's output, with the D6 permute fix)."""
        b = img.shape[0]
        x = img.reshape(b, self.size, self.size, 1)
        mask = (x == 0).reshape(b, -1)  # zero pixels are padding keys
        logits = self.perceiver(x, mask)  # (B, H*W, 3)
        return logits.permute(0, 2, 1)

    def sparse_hidden(self, values, index, kmask, qidx):
        """Decoder output ``(B, K', C)`` at output pixels ``qidx``, from the non-zero pixels only."""
        from .. import ops

        enc, dec = self.perceiver.encoder, self.perceiver.decoder
        if ops.use_hip(enc.latent):  # PE rows read at `index` inside the K/V projection kernels
            lat = ops.fused.encode_sparse(enc, values, index, kmask)
        else:
            lat = enc.forward_inputs(sparse_inputs(enc.input_adapter, values, index), kmask)
        return dec.hidden_at(lat, qidx)

    def sparse_logits(self, values, index, kmask, qidx):
        """Logits ``(B, K', 3)`` at output pixels ``qidx`` from the non-zero pixels only."""
        return self.perceiver.decoder.output_adapter.linear(self.sparse_hidden(values, index, kmask, qidx))

    def sparse_loss(self, batch, weights: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        """``(loss, {acc, acc1, acc2})`` for a :func:`data.lartpc.sparse_collate` batch: the
        weighted mean cross-entropy of the dense model (ignored slots are -100) and the
        reference's per-class accuracies, as device tensors.  On the GPU the 3-way head, the
        loss and the accuracies are one fused kernel each way (``ops/pixel_head.py``)."""
        from ..ops.pixel_head import pixel_ce

        values, index, kmask, qidx, qlab = batch
        h = self.sparse_hidden(values, index, kmask, qidx)
        return pixel_ce(h, self.perceiver.decoder.output_adapter.linear, qlab, weights)


def accuracies(pred: torch.Tensor, lab: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Per-class accuracies of the reference (``run.py:190-206``) as device tensors: over labelled
    pixels (label > 0), tracks (1) and showers (2); 0 where a class is absent."""
    out = {}
    for name, sel in (("acc", lab > 0), ("acc1", lab == 1), ("acc2", lab == 2)):
        n = sel.sum()
        hit = ((pred == lab) & sel).sum()
        out[name] = torch.where(n > 0, hit.float() / n.clamp(min=1).float(), torch.zeros((), device=lab.device))
    return out


def class_weights(device, weights: Sequence[float] = CLASS_WEIGHTS) -> torch.Tensor:
    return torch.tensor(list(weights), dtype=torch.float32, device=device)
