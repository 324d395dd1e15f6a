"""Import-compatible surface of the reference package ``perceiver`` (``perceiver/__init__.py``):
``from perceiver import LitMaskedLanguageModel, PerceiverIO, ...`` keeps working; everything is
implemented in :mod:`perceiver_io_amd`."""
from perceiver_io_amd.models.adapters import *  # noqa: F401,F403
from perceiver_io_amd.models.perceiver import PerceiverDecoder, PerceiverEncoder, PerceiverIO, PerceiverMLM, TextMasking  # noqa: F401
from perceiver_io_amd.tasks import LitImageClassifier, LitMaskedLanguageModel, LitTextClassifier  # noqa: F401
