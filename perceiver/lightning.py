"""``perceiver.lightning`` compatibility module (reference ``perceiver/lightning.py``)."""
from perceiver_io_amd.tasks import (LitClassifier, LitImageClassifier, LitMaskedLanguageModel, LitModel,  # noqa: F401
                                    LitTextClassifier)
