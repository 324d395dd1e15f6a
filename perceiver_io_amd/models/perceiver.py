"""Perceiver IO encoder / decoder / MLM models.

Reference parity (``perceiver/model.py``):
  * ``PerceiverEncoder`` — ``model.py:119-189``: learned latent (N, C) repeated over the
    batch, ``layer_1`` then the *same* ``layer_n`` applied ``num_layers-1`` times
    (weight sharing); returns ``(latent, pad_mask)``.
  * ``PerceiverDecoder`` — ``model.py:192-237``: learned output query (K, C_out), one
    unmasked cross-attention layer over the latents, then the output adapter.
  * ``TextMasking``      — ``model.py:240-293``: BERT 80/10/10 masking.  Implemented
    out-of-place and without host syncs (fixes D4 and the two ``nonzero``/``sum``
    syncs of the reference).
  * ``PerceiverMLM``     — ``model.py:296-318`` with defect D2 fixed (the encoder
    tuple is unpacked before the decoder).
  * ``PerceiverIO``      — ``model.py:321-325``; children stay ``0``/``1`` for
    checkpoint keys, with ``.encoder``/``.decoder`` aliases (defect D3 fixed).

MI355X-specific additions (same maths, less work):
  * ``PerceiverMLM.loss`` decodes every query but runs the 10k-way vocab projection
    and cross-entropy only on the ~15 % selected positions: decoder
    queries never interact, so loss and gradients are identical to the reference's
    full ``(B, V, L)`` cross-entropy.
  * ``PerceiverEncoder`` computes the input-side kv-LayerNorm + K/V projection of the
    weight-shared ``layer_n`` once per forward instead of ``num_layers-1`` times on the
    fused path (SURVEY K-06).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..parallel.reducer import bucket_ready_point, ready_point_armed
from ..utils.tokenizer import MASK_TOKEN, SPECIAL_TOKENS, UNK_TOKEN
from .adapters import InputAdapter, OutputAdapter
from .blocks import Sequential, cross_attention_layer, init_latent_, self_attention_block


class PerceiverEncoder(nn.Module):
    def __init__(self,
                 input_adapter: InputAdapter,
                 latent_shape: Tuple[int, int],
                 num_layers: int,
                 num_cross_attention_heads: int = 4,
                 num_self_attention_heads: int = 4,
                 num_self_attention_layers_per_block: int = 2,
                 dropout: float = 0.0):
        super().__init__()
        self.input_adapter = input_adapter
        self.num_layers = num_layers
        self.latent_shape = tuple(latent_shape)
        c = latent_shape[1]

        def perceiver_layer():
            return Sequential(
                cross_attention_layer(c, input_adapter.num_input_channels, num_cross_attention_heads, dropout),
                self_attention_block(num_self_attention_layers_per_block, c, num_self_attention_heads, dropout),
            )

        self.layer_1 = perceiver_layer()
        if num_layers > 1:
            self.layer_n = perceiver_layer()  # applied recurrently (weight sharing)
        self.latent = nn.Parameter(torch.empty(*latent_shape))
        init_latent_(self.latent)

    def layers(self):
        """The layer sequence actually executed (``layer_n`` repeated)."""
        if self.num_layers <= 1:
            return [self.layer_1]
        return [self.layer_1] + [self.layer_n] * (self.num_layers - 1)

    def forward(self, x, pad_mask=None, attn_mask=None):
        b = x.shape[0]
        if attn_mask is None and ops.use_hip(self.latent):
            return ops.fused.encoder_forward(self, x, pad_mask), pad_mask
        return self.forward_inputs(self.input_adapter(x), pad_mask, attn_mask), pad_mask

    def forward_inputs(self, x_in, pad_mask=None, attn_mask=None):
        """Latents for already adapted inputs ``x_in`` (B, M, Kin), bypassing the input adapter
        (used for sparse image inputs: the adapter's rows gathered at the non-zero pixels)."""
        if attn_mask is None and ops.use_hip(self.latent):
            return ops.fused.encode_inputs(self, x_in, pad_mask)
        x_latent = self.latent.unsqueeze(0).expand(x_in.shape[0], -1, -1)
        layers = self.layers()
        for i, layer in enumerate(layers):
            if i == 1:  # DDP: layer_n's gradients are final here (parallel/reducer.py)
                x_latent = bucket_ready_point(x_latent, self, "layer_n")
            if i == 0 and len(layers) > 1:  # DDP: layer_1's self-attention block gradients final here
                x_latent = layer[0](x_latent, x_in, pad_mask, attn_mask)
                x_latent = layer[1](bucket_ready_point(x_latent, self, "layer_1_sa"))
                continue
            x_latent = layer(x_latent, x_in, pad_mask, attn_mask)
        return x_latent


class PerceiverDecoder(nn.Module):
    def __init__(self,
                 output_adapter: OutputAdapter,
                 latent_shape: Tuple[int, int],
                 num_cross_attention_heads: int = 4,
                 dropout: float = 0.0):
        super().__init__()
        num_latent_channels = latent_shape[1]
        num_output_channels = output_adapter.output_shape[-1]
        self.output_adapter = output_adapter
        self.latent_shape = tuple(latent_shape)
        self.cross_attention = cross_attention_layer(num_q_channels=num_output_channels,
                                                     num_kv_channels=num_latent_channels,
                                                     num_heads=num_cross_attention_heads,
                                                     dropout=dropout)
        self.output = nn.Parameter(torch.empty(*output_adapter.output_shape))
        init_latent_(self.output)

    def check_latent(self, x):
        d = tuple(x.shape[1:])
        if d != self.latent_shape:
            raise ValueError(f"Latent shape {d} different from required shape {self.latent_shape}")

    def hidden(self, x, num_queries: Optional[int] = None):
        """Decoder output before the adapter, ``(B, K, C_out)``; optionally only the
        first ``num_queries`` queries (queries are independent of each other)."""
        x = bucket_ready_point(x, self, "decoder")  # DDP: decoder grads final here (parallel/reducer.py)
        self.check_latent(x)
        q = (self.output if num_queries is None else self.output[:num_queries]).unsqueeze(0)
        ca = self.cross_attention
        if ca._fusable(x, None) and ops.fused.can_fuse(ca, x):
            # one query stream broadcast over the batch inside the fused kernels: the query
            # gradient comes back summed over the batch (no expand / slice backward glue)
            return ca(q, x)
        return ca(q.expand(x.shape[0], -1, -1), x)

    def loss(self, x_latent, labels):
        """Mean cross-entropy of the output adapter's logits against ``labels`` (classification
        adapters); on the GPU through the fused vocab-projection + CE kernels (no logits tensor)."""
        return ops.mlm_head.classification_loss(self, x_latent, labels)

    def hidden_at(self, x, idx):
        """Decoder output at output-query rows ``idx`` (B, K') only, ``(B, K', C_out)``: queries
        never interact, so this equals ``hidden(x)`` gathered at ``idx``.  The gather's backward
        adds straight into the query parameter's gradient rows."""
        from ..ops.mlm_head import _GatherQueries

        x = bucket_ready_point(x, self, "decoder")
        self.check_latent(x)
        q = _GatherQueries.apply(self.output, idx.reshape(-1)).view(idx.shape[0], idx.shape[1], -1)
        return self.cross_attention(q, x)

    def forward(self, x, pad_mask=None):
        return self.output_adapter(self.hidden(x))


class PerceiverIO(Sequential):
    def __init__(self, encoder: PerceiverEncoder, decoder: PerceiverDecoder):
        super().__init__(encoder, decoder)

    def loss(self, x, labels, pad_mask=None):
        """Training loss of a classifier: ``cross_entropy(self(x, pad_mask), labels)`` computed
        through the decoder's fused head (same value and gradients)."""
        look = ops.fused._LOOKAHEAD
        # on the fused path the encoder's last per-sample block also projects the decoder's K/V
        # (and runs that projection's backward, unless a DDP ready point on the decoder input needs
        # the decoder's gradients final before the encoder backward)
        look["want_kv"] = (ops.fused.decoder_kv_lookahead(
            self.decoder.cross_attention, sample_block=True,
            backward=not ready_point_armed(self.decoder, "decoder")) if ops.use_hip(x) else None)
        try:
            x_latent, _ = self.encoder(x, pad_mask)
            return self.decoder.loss(x_latent, labels)
        finally:
            look["want_kv"] = look["have_q"] = None

    @property
    def encoder(self) -> PerceiverEncoder:
        return self[0]

    @property
    def decoder(self) -> PerceiverDecoder:
        return self[1]


class TextMasking(nn.Module):
    """BERT masking: of the non-special tokens (not UNK, not PAD) select 15 %; of those
    80 % → ``[MASK]``, 10 % → random non-special id, 10 % unchanged.  Labels are the
    original ids at selected positions and -100 elsewhere."""

    def __init__(self, vocab_size: int, unk_token_id: int = 1, mask_token_id: int = 2,
                 num_special_tokens: int = len(SPECIAL_TOKENS), mask_p: float = 0.15):
        super().__init__()
        self.vocab_size = vocab_size
        self.unk_token_id = unk_token_id
        self.mask_token_id = mask_token_id
        self.num_special_tokens = num_special_tokens
        self.mask_p = mask_p

    @staticmethod
    def create(tokenizer, **kwargs):
        return TextMasking(vocab_size=tokenizer.get_vocab_size(),
                           unk_token_id=tokenizer.token_to_id(UNK_TOKEN),
                           mask_token_id=tokenizer.token_to_id(MASK_TOKEN),
                           num_special_tokens=len(SPECIAL_TOKENS), **kwargs)

    def forward(self, x, pad_mask=None, generator: Optional[torch.Generator] = None):
        if ops.get_backend() == "reference":
            return self._reference_masking(x, pad_mask)
        return ops.masking.text_masking(x, pad_mask, self.vocab_size, self.unk_token_id, self.mask_token_id,
                                        self.num_special_tokens, self.mask_p, generator=generator)

    def _reference_masking(self, x, pad_mask):
        """The reference's compute pattern (boolean-index scatter, ``randint(size=sum)`` —
        two device→host syncs), out of place.  Used only by the ``reference`` backend."""
        x = x.clone()
        labels = x.clone()
        special = x == self.unk_token_id
        if pad_mask is not None:
            special |= pad_mask
        sel = (torch.rand_like(x, dtype=torch.float) < self.mask_p) & ~special
        sel1 = sel & (torch.rand_like(x, dtype=torch.float) < 0.9)
        sel2 = sel1 & (torch.rand_like(x, dtype=torch.float) < 1 / 9)
        x[sel1] = self.mask_token_id
        x[sel2] = torch.randint(self.num_special_tokens, self.vocab_size, size=(int(sel2.sum()),), device=x.device)
        labels[~sel] = -100
        return x, labels


class PerceiverMLM(nn.Module):
    def __init__(self, encoder: PerceiverEncoder, decoder: PerceiverDecoder, masking: TextMasking):
        super().__init__()
        self.encoder = encoder
        self.decoder = decoder
        self.masking = masking

    def forward(self, x_input, pad_mask=None, masking: bool = True):
        l = x_input.shape[1]
        if masking:
            x_masked, x_labels = self.masking(x_input, pad_mask)
        else:
            x_masked, x_labels = x_input, None
        x_latent, _ = self.encoder(x_masked, pad_mask)
        x_logits = self.decoder.output_adapter(self.decoder.hidden(x_latent, num_queries=l))
        return x_logits, x_labels

    def loss(self, x_input, pad_mask=None, labels=None, x_masked=None):
        """Masked-token cross-entropy (mean over selected positions) without
        materialising the ``(B, L, V)`` logits.  ``labels``/``x_masked`` may be given
        to replay a fixed masking."""
        l = x_input.shape[1]
        if labels is None:
            x_masked, labels = self.masking(x_input, pad_mask)
        if ops.get_backend() == "reference":
            x_latent, _ = self.encoder(x_masked, pad_mask)
            # reference compute: all K queries decoded, full (B, V, L) logits, CE with ignore_index
            logits = self.decoder(x_latent)[:, :l, :]
            return torch.nn.functional.cross_entropy(logits.transpose(1, 2), labels, ignore_index=-100)
        look = ops.fused._LOOKAHEAD
        # on the fused path the encoder's last kernel also projects the decoder's K/V
        look["want_kv"] = (ops.fused.decoder_kv_lookahead(self.decoder.cross_attention)
                           if ops.use_hip(x_masked) else None)
        try:
            x_latent, _ = self.encoder(x_masked, pad_mask)
            return ops.mlm_head.masked_decode_loss(self.decoder, x_latent, labels, p=self.masking.mask_p)
        finally:
            look["want_kv"] = look["have_q"] = None
