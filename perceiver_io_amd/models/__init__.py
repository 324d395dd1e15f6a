"""Model families: Perceiver IO encoder/decoder, adapters, MLM, task modules."""
from .adapters import (ClassificationOutputAdapter, ImageInputAdapter, InputAdapter, OutputAdapter,
                       SemanticSegOutputAdapter, TextInputAdapter, TextOutputAdapter, fourier_position_encoding)
from .blocks import (CrossAttention, MultiHeadAttention, Residual, SelfAttention, Sequential, cross_attention_layer, mlp,
                     self_attention_block, self_attention_layer)
from .perceiver import PerceiverDecoder, PerceiverEncoder, PerceiverIO, PerceiverMLM, TextMasking

__all__ = [
    "InputAdapter", "OutputAdapter", "ImageInputAdapter", "TextInputAdapter", "ClassificationOutputAdapter",
    "SemanticSegOutputAdapter", "TextOutputAdapter", "fourier_position_encoding", "Sequential", "mlp", "Residual",
    "MultiHeadAttention", "CrossAttention", "SelfAttention", "cross_attention_layer", "self_attention_layer",
    "self_attention_block", "PerceiverEncoder", "PerceiverDecoder", "PerceiverIO", "PerceiverMLM", "TextMasking",
]
