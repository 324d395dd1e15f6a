"""Loader for the in-tree HIP extension ``perceiver_io_amd/_C*.so``.

The extension is built by :mod:`perceiver_io_amd.csrc.build` (``hipcc
--offload-arch=gfx950``), kept in-tree so it travels with the repo snapshot to the
GPU box.  There is deliberately no JIT path and no PyTorch fallback once a GPU
tensor reaches a fused op: a missing extension is an error.
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    try:
        # PERCEIVER_CHECKED=1: the checked build (device-side index validation, see csrc/build.py)
        name = "perceiver_io_amd._C_check" if os.environ.get("PERCEIVER_CHECKED", "0") not in ("", "0") \
            else "perceiver_io_amd._C"
        _mod = importlib.import_module(name)
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _mod


def available() -> bool:
    return _load() is not None


def require():
    m = _load()
    if m is None:
        raise RuntimeError(
            "perceiver_io_amd HIP extension (_C) is not built/loadable: "
            f"{_err!r}. Build it with `python -m perceiver_io_amd.csrc.build` "
            "(hipcc --offload-arch=gfx950) or select the eager backend with "
            "PERCEIVER_BACKEND=torch.")
    return m


def __getattr__(name):  # ext.<kernel>(...) convenience
    if name.startswith("__"):
        raise AttributeError(name)
    return getattr(require(), name)
