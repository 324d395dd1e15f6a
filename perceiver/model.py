"""``perceiver.model`` compatibility module (reference ``perceiver/model.py``)."""
from perceiver_io_amd.models.blocks import (CrossAttention, MultiHeadAttention, Residual, SelfAttention,  # noqa: F401
                                            Sequential, cross_attention_layer, mlp, self_attention_block,
                                            self_attention_layer)
from perceiver_io_amd.models.perceiver import (PerceiverDecoder, PerceiverEncoder, PerceiverIO, PerceiverMLM,  # noqa: F401
                                               TextMasking)
