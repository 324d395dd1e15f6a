"""Lightning-layout checkpoint I/O.

Top-level keys written: ``epoch``, ``global_step``, ``pytorch-lightning_version``,
``state_dict``, ``callbacks``, ``optimizer_states``, ``lr_schedulers``, ``hparams_name``,
``hyper_parameters`` — what PL 1.5 writes and what ``load_from_checkpoint`` /
``--trainer.resume_from_checkpoint`` read (reference ``lightning.py:144-149``,
``trainer.yaml:54``).  Everything written is reduced to tensors and plain Python values so
every checkpoint loads with ``torch.load(..., weights_only=True)``; nothing is ever fully
unpickled.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, Optional

import torch

PL_VERSION = "1.5.10"
TAG = "perceiver_io_amd"


def _plain(obj):
    """Tensors and plain Python containers/scalars only (safe for ``weights_only``)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {(k if isinstance(k, (str, int)) else str(k)): _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_plain(v) for v in obj)
    if isinstance(obj, (str, int, float, bool)) or obj is None:
        return obj
    return str(obj)


def make_checkpoint(model, epoch: int, global_step: int, optimizers=(), schedulers=(), callbacks: Optional[Dict] = None):
    sd = OrderedDict((k, v.detach().cpu()) for k, v in model.state_dict().items())
    return {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": PL_VERSION,
        "state_dict": sd,
        "callbacks": _plain(callbacks or {}),
        "optimizer_states": [_plain(o.state_dict()) for o in optimizers],
        "lr_schedulers": [_plain(s.state_dict()) for s in schedulers],
        "hparams_name": "kwargs",
        "hyper_parameters": _plain(dict(getattr(model, "hparams", {}) or {})),
        TAG: {"format": 1},
    }


def save_checkpoint(ckpt: Dict[str, Any], path: str):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    """Safe load only (``weights_only=True``); a file that needs arbitrary unpickling is refused."""
    return torch.load(path, map_location=map_location, weights_only=True)
