"""LightningModule-compatible base (PyTorch-Lightning is not part of this stack).

Provides the pieces of the ``pl.LightningModule`` surface the reference's task modules use
(``perceiver/lightning.py``): ``save_hyperparameters`` capturing every ``__init__`` argument up
the subclass chain (``lightning.py:42``), ``hparams``, ``log``, ``trainer``/``device``/
``logger`` properties, ``configure_optimizers`` from ``{class_path, init_args}`` dicts
(``lightning.py:44-55``) and ``load_from_checkpoint`` that rebuilds via
``cls(**hyper_parameters)`` then loads the ``state_dict`` strictly (``lightning.py:145,148``).
"""
from __future__ import annotations

import importlib
import inspect
from typing import Any, Dict, Optional

import torch
import torch.nn as nn


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def import_class(path: str):
    mod, _, name = path.rpartition(".")
    aliases = {
        "pytorch_lightning.callbacks.lr_monitor": "perceiver_io_amd.train.callbacks",
        "pytorch_lightning.callbacks.model_checkpoint": "perceiver_io_amd.train.callbacks",
        "pytorch_lightning.callbacks": "perceiver_io_amd.train.callbacks",
    }
    mod = aliases.get(mod, mod)
    return getattr(importlib.import_module(mod), name)


def instantiate_class(args, init: Dict[str, Any]):
    """``instantiate_class(args, {"class_path": ..., "init_args": {...}})`` (LightningCLI helper)."""
    cls = import_class(init["class_path"])
    kwargs = dict(init.get("init_args", {}) or {})
    if not isinstance(args, tuple):
        args = (args,)
    return cls(*args, **kwargs)


def _collect_init_args(obj) -> Dict[str, Any]:
    """Walk the call stack of the ``__init__`` chain of ``obj`` and merge their arguments
    (outermost subclass wins), flattening ``**kwargs``."""
    frame = inspect.currentframe()
    out: Dict[str, Any] = {}
    chain = []
    f = frame.f_back
    while f is not None:
        if f.f_code.co_name == "__init__" and f.f_locals.get("self") is obj:
            chain.append(f)
        f = f.f_back
    for f in reversed(chain):  # outermost first, inner frames complete missing values
        code = f.f_code
        names = code.co_varnames[: code.co_argcount + code.co_kwonlyargcount]
        loc = f.f_locals
        for n in names:
            if n == "self":
                continue
            if n not in out and n in loc:
                out[n] = loc[n]
        if code.co_flags & inspect.CO_VARKEYWORDS:
            kw_name = code.co_varnames[code.co_argcount + code.co_kwonlyargcount + (1 if code.co_flags & inspect.CO_VARARGS else 0)]
            for k, v in (loc.get(kw_name) or {}).items():
                out.setdefault(k, v)
    del frame
    # drop *args / **kwargs containers themselves
    return {k: v for k, v in out.items() if k not in ("args", "kwargs")}


class LitModuleBase(nn.Module):
    def __init__(self):
        super().__init__()
        self._hparams = AttributeDict()
        self._trainer = None
        self._logged: Dict[str, Any] = {}

    # -- hyper-parameters -----------------------------------------------------------------
    def save_hyperparameters(self):
        args = _collect_init_args(self)
        self._hparams = AttributeDict(args)

    @property
    def hparams(self) -> AttributeDict:
        return self._hparams

    # -- trainer hooks ---------------------------------------------------------------------
    @property
    def trainer(self):
        return self._trainer

    @property
    def logger(self):
        return self._trainer.logger if self._trainer is not None else None

    @property
    def device(self) -> torch.device:
        for p in self.parameters():
            return p.device
        return torch.device("cpu")

    @property
    def global_step(self) -> int:
        return self._trainer.global_step if self._trainer is not None else 0

    def log(self, name: str, value, prog_bar: bool = False, on_step: Optional[bool] = None,
            on_epoch: Optional[bool] = None, sync_dist: bool = False, **_):
        if self._trainer is not None:
            self._trainer._log(name, value, prog_bar=prog_bar, on_step=on_step, on_epoch=on_epoch, sync_dist=sync_dist)

    def configure_optimizers(self):
        raise NotImplementedError

    def on_validation_epoch_end(self) -> None:
        pass

    def graph_batch(self, batch):
        """Canonicalise a training batch before a hipGraph-captured step (graphs are cached
        per batch shape, train/engine.py).  Identity here; text modules bucket lengths."""
        return batch

    # -- checkpoints ----------------------------------------------------------------------
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: str, map_location=None, strict: bool = True, **overrides):
        from .checkpoint import load_checkpoint

        ckpt = load_checkpoint(checkpoint_path, map_location=map_location or "cpu")
        hp = dict(ckpt.get("hyper_parameters", {}))
        hp.update(overrides)
        model = cls(**hp)
        model.load_state_dict(ckpt["state_dict"], strict=strict)
        return model
