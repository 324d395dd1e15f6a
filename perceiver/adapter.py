"""``perceiver.adapter`` compatibility module (reference ``perceiver/adapter.py``)."""
from perceiver_io_amd.models.adapters import (ClassificationOutputAdapter, ImageInputAdapter, InputAdapter,  # noqa: F401
                                              OutputAdapter, SemanticSegOutputAdapter, TextInputAdapter,
                                              TextOutputAdapter)
