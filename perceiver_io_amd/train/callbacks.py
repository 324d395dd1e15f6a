"""Trainer callbacks with the reference's defaults (``scripts/trainer.yaml:5-14``):
``LearningRateMonitor(logging_interval='step')`` and
``ModelCheckpoint(monitor='val_loss', filename='{epoch:03d}-{val_loss:.3f}', mode='min')``
saving into ``<log_dir>/checkpoints/`` on rank 0 (``README.md:78,97`` paths)."""
from __future__ import annotations

import math
import os
import re
from typing import Any, Dict, Optional


class Callback:
    def on_fit_start(self, trainer, module): ...
    def on_train_batch_end(self, trainer, module): ...
    def on_validation_end(self, trainer, module): ...
    def on_train_epoch_end(self, trainer, module): ...
    def on_fit_end(self, trainer, module): ...

    def state_key(self) -> str:
        return type(self).__name__

    def state_dict(self) -> Dict[str, Any]:
        return {}

    def load_state_dict(self, sd: Dict[str, Any]): ...


class LearningRateMonitor(Callback):
    def __init__(self, logging_interval: Optional[str] = None, log_momentum: bool = False):
        self.logging_interval = logging_interval or "step"
        self.log_momentum = log_momentum

    def _log(self, trainer):
        for i, opt in enumerate(trainer.optimizers):
            for j, g in enumerate(opt.param_groups):
                name = f"lr-{type(opt).__name__}" + (f"/pg{j + 1}" if len(opt.param_groups) > 1 else "")
                trainer.log_scalars({name: g["lr"]})
                if self.log_momentum and "betas" in g:
                    trainer.log_scalars({name.replace("lr-", "lr-momentum-"): g["betas"][0]})

    def on_train_batch_end(self, trainer, module):
        if self.logging_interval == "step" and trainer.global_step % trainer.log_every_n_steps == 0:
            self._log(trainer)

    def on_train_epoch_end(self, trainer, module):
        if self.logging_interval == "epoch":
            self._log(trainer)


class ModelCheckpoint(Callback):
    def __init__(self, dirpath: Optional[str] = None, filename: Optional[str] = None, monitor: Optional[str] = None,
                 verbose: bool = False, save_last: Optional[bool] = None, save_top_k: int = 1, mode: str = "min",
                 every_n_train_steps: Optional[int] = None, every_n_epochs: Optional[int] = None, **_):
        self.dirpath = dirpath
        self.filename = filename
        self.monitor = monitor
        self.save_last = save_last
        self.save_top_k = save_top_k
        self.mode = mode
        self.every_n_train_steps = every_n_train_steps
        self.best_model_score: Optional[float] = None
        self.best_model_path: str = ""
        self.last_model_path: str = ""
        self.best_k_models: Dict[str, float] = {}
        self.verbose = verbose

    def state_key(self) -> str:
        return f"ModelCheckpoint{{'monitor': {self.monitor!r}, 'mode': {self.mode!r}}}"

    def state_dict(self):
        return {"monitor": self.monitor, "best_model_score": self.best_model_score,
                "best_model_path": self.best_model_path, "last_model_path": self.last_model_path,
                "best_k_models": dict(self.best_k_models), "dirpath": self.dirpath}

    def load_state_dict(self, sd):
        self.best_model_score = sd.get("best_model_score")
        self.best_model_path = sd.get("best_model_path", "")
        self.best_k_models = dict(sd.get("best_k_models", {}))

    def _dir(self, trainer) -> str:
        if self.dirpath:
            return os.path.abspath(self.dirpath)
        base = trainer.logger.log_dir if trainer.logger is not None else trainer.default_root_dir
        return os.path.abspath(os.path.join(base, "checkpoints"))

    def format_name(self, metrics: Dict[str, float], epoch: int, step: int) -> str:
        fn = self.filename or ("{epoch}-{step}" if self.monitor is None else "{epoch}-{step}")
        groups = re.findall(r"\{([^{}:]+)(:[^{}]*)?\}", fn)
        vals = {"epoch": epoch, "step": step, **metrics}
        for name, fmt in groups:
            v = vals.get(name, 0)
            spec = "{" + (fmt or "") + "}"
            spec = "{:" + fmt[1:] + "}" if fmt else "{}"
            fn = fn.replace("{" + name + (fmt or "") + "}", f"{name}=" + spec.format(v))
        return fn + ".ckpt"

    def _better(self, v: float, ref: Optional[float]) -> bool:
        if ref is None:
            return True
        return v < ref if self.mode == "min" else v > ref

    def _save(self, trainer, module, path: str):
        trainer.save_checkpoint(path)

    def on_validation_end(self, trainer, module):
        if trainer.sanity_checking or not trainer.is_global_zero_or_all():
            return
        metrics = trainer.callback_metrics
        epoch, step = trainer.current_epoch, trainer.global_step
        d = self._dir(trainer)
        if self.monitor is None:
            path = os.path.join(d, self.format_name(metrics, epoch, step))
            self._save(trainer, module, path)
            self.last_model_path = path
            return
        if self.monitor not in metrics:
            return
        v = float(metrics[self.monitor])
        if math.isnan(v):
            return
        if self.save_top_k == 0:
            return
        worst_path = None
        if self.save_top_k > 0 and len(self.best_k_models) >= self.save_top_k:
            worst_path = max(self.best_k_models, key=self.best_k_models.get) if self.mode == "min" else \
                min(self.best_k_models, key=self.best_k_models.get)
            if not self._better(v, self.best_k_models[worst_path]):
                return
        path = os.path.join(d, self.format_name(metrics, epoch, step))
        self._save(trainer, module, path)
        self.best_k_models[path] = v
        if worst_path is not None and worst_path != path:
            self.best_k_models.pop(worst_path, None)
            if trainer.is_global_zero and os.path.exists(worst_path):
                os.remove(worst_path)
        best = min(self.best_k_models, key=self.best_k_models.get) if self.mode == "min" else \
            max(self.best_k_models, key=self.best_k_models.get)
        self.best_model_path, self.best_model_score = best, self.best_k_models[best]
        if self.save_last:
            last = os.path.join(d, "last.ckpt")
            self._save(trainer, module, last)
            self.last_model_path = last


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "val_loss", patience: int = 3, mode: str = "min", min_delta: float = 0.0, **_):
        self.monitor, self.patience, self.mode, self.min_delta = monitor, patience, mode, min_delta
        self.best, self.wait = None, 0

    def on_validation_end(self, trainer, module):
        if trainer.sanity_checking or self.monitor not in trainer.callback_metrics:
            return
        v = float(trainer.callback_metrics[self.monitor])
        improved = self.best is None or (v < self.best - self.min_delta if self.mode == "min" else v > self.best + self.min_delta)
        if improved:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                trainer.should_stop = True
