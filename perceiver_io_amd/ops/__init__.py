"""Op layer: hand-written HIP/CDNA4 kernels (``perceiver_io_amd/csrc``) behind
autograd Functions, plus the eager PyTorch oracle used on CPU and in tests.

Backend selection (``PERCEIVER_BACKEND`` env or :func:`set_backend`):
  * ``auto``  — HIP kernels for CUDA(HIP) tensors, eager PyTorch on CPU.  On a GPU
    box a missing/broken extension raises instead of silently falling back.
  * ``hip``   — force the kernels (error if unavailable).
  * ``torch`` — eager PyTorch everywhere (this framework's own eager oracle).
  * ``reference`` — eager PyTorch with the reference's exact compute: ``nn.MultiheadAttention``
    math (``F.multi_head_attention_forward``, need_weights=True), full ``(B, V, L)`` logits
    cross-entropy and sync-ing boolean-index masking.  Used to measure the baseline.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch

from . import ext  # noqa: F401  (extension loader)

_BACKEND = os.environ.get("PERCEIVER_BACKEND", "auto")
_VALID = ("auto", "hip", "torch", "reference")


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in _VALID:
        raise ValueError(f"backend must be one of {_VALID}, got {name!r}")
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


@contextmanager
def backend(name: str):
    prev = get_backend()
    set_backend(name)
    try:
        yield
    finally:
        set_backend(prev)


_DETERMINISTIC = [False]


def set_deterministic(flag: bool) -> None:
    """Deterministic mode (trainer ``deterministic=True``): every kernel reduction
    that would use fp32 atomics with several writers per address runs as a fixed-order split
    reduction, so identical runs give bitwise-identical parameters."""
    _DETERMINISTIC[0] = bool(flag)
    if ext.available():
        ext.require().set_deterministic(bool(flag))


def deterministic() -> bool:
    return _DETERMINISTIC[0]


def check_device_errors(reset: bool = True) -> None:
    """Read the kernels' sticky device error words (one host sync) and raise on any.

    * ``csrc/persist.hip`` ``sa_block_fwd``: a bounded spin that timed out (bit 0: a tile gave up
      waiting for its sample's next-layer Q/K/V rows and computed on whatever was there) or an
      invalid tile ticket (bit 1).  The launch finishes either way (no GPU hang); this turns the
      corrupted forward into an error instead of silent training on garbage.
    * checked builds (``PERCEIVER_CHECKED=1``): the index-validation words — token ids, gather
      rows and class labels outside their tables (the kernels clamped / skipped the access).
      Outside a graph capture every checked launch raises at once (``checked_sync``); inside a
      replayed hipGraph nothing can.

    Called by the Trainer at every logging step and at the end of ``fit`` and by ``bench.py``
    after its timed loop (SURVEY §5.3 failure detection)."""
    if not ext.available() or not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    K = ext.require()
    e = int(K.persist_errors(reset))
    if e:
        what = []
        if e & 1:
            what.append("a bounded spin timed out: a tile computed on rows its sample had not published")
        if e & 2:
            what.append("a workgroup drew a tile ticket outside the grid")
        raise RuntimeError(f"sa_block_fwd_kernel (csrc/persist.hip) device error word {e:#x}: " + "; ".join(what)
                           + ".  The persistent self-attention block forward's results of that step are invalid")
    if K.checked_build():
        c = int(K.check_errors(reset))
        if c:
            raise RuntimeError(f"checked build: out-of-range indices seen on the device (error bits {c:#x}: "
                               "1 token id >= vocab, 2 gather row out of range, 4 label outside [0, V) and != -100, "
                               "8 PE row index outside the position-encoding table)")


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` should be processed by the HIP kernels."""
    if _BACKEND in ("torch", "reference") or not t.is_cuda:
        return False
    ext.require()  # raises loudly if the extension is missing on a GPU
    return True


from . import attention, fused, masking, mlm_head, optim  # noqa: E402,F401
