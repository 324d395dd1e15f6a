"""``perceiver.tokenizer`` compatibility module (reference ``perceiver/tokenizer.py``)."""
from perceiver_io_amd.utils.tokenizer import *  # noqa: F401,F403
