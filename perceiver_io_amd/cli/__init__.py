"""LightningCLI-compatible command line (reference ``scripts/cli.py``).

    python scripts/mlm.py fit --model.dropout=0.0 --data=IMDBDataModule --data.max_seq_len=512 \\
        --data.batch_size=64 --optimizer.lr=0.003 --optimizer.weight_decay=0.0 \\
        --lr_scheduler.pct_start=0.1 --trainer.accelerator=gpu --trainer.devices=-1 --trainer.max_steps=50000

Surface reproduced: subcommands ``fit|validate|test``; dotted flags ``--model.* --data=<Class>
--data.* --trainer.* --optimizer.* --lr_scheduler.* --logger.* --experiment --config
--print_config --seed_everything``; per-subcommand default YAML (``scripts/trainer.yaml``);
parse-time links (``trainer.default_root_dir→logger.save_dir``, ``experiment→logger.name``,
``trainer.max_steps→lr_scheduler.total_steps``, ``optimizer.lr→lr_scheduler.max_lr``) and
instantiate-time links (``data.vocab_size/max_seq_len/num_classes/image_shape→model.*``);
``set_defaults``; optimizer / scheduler carried as ``{class_path, init_args}`` into the model;
``config.yaml`` saved into the log directory (overwrite).  Values are parsed with
``yaml.safe_load`` (lists, bools, numbers, null).

Multi-GPU: ``--trainer.devices=N|-1`` with a GPU accelerator re-launches the script as one
process per GPU (``parallel/launch.py``) before anything touches the GPU.
"""
from __future__ import annotations

import copy
import inspect
import os
import sys
from typing import Any, Dict, List, Optional

import yaml

SUBCOMMANDS = ("fit", "validate", "test")


def _parse_value(s: str):
    try:
        return yaml.safe_load(s)
    except yaml.YAMLError:
        return s


def _set(cfg: Dict, dotted: str, value):
    parts = dotted.split(".")
    d = cfg
    for p in parts[:-1]:
        if not isinstance(d.get(p), dict):
            d[p] = {} if d.get(p) is None or not isinstance(d.get(p), str) else {"class": d[p]}
        d = d[p]
    d[parts[-1]] = value


def _get(cfg: Dict, dotted: str, default=None):
    d = cfg
    for p in dotted.split("."):
        if not isinstance(d, dict) or p not in d:
            return default
        d = d[p]
    return d


def _merge(dst: Dict, src: Dict):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)


def _signature_defaults(cls, skip=("self",)) -> Dict[str, Any]:
    out = {}
    for name, p in inspect.signature(cls.__init__).parameters.items():
        if name in skip or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
            continue
        out[name] = None if p.default is inspect.Parameter.empty else p.default
    return out


class CLIParser:
    """The subset of ``LightningArgumentParser`` the reference scripts use."""

    def __init__(self):
        self.links: List[tuple] = []
        self.defaults: Dict[str, Any] = {}
        self.optimizer = None
        self.lr_scheduler = None
        self.class_args: Dict[str, Any] = {}
        self.extra_args: Dict[str, Any] = {}

    def link_arguments(self, source: str, target: str, compute_fn=None, apply_on: str = "parse"):
        self.links.append((source, target, compute_fn, apply_on))

    def set_defaults(self, d: Dict[str, Any]):
        self.defaults.update(d)

    def add_optimizer_args(self, cls, link_to: str = "model.optimizer_init", nested_key: str = "optimizer"):
        self.optimizer = (cls, link_to, nested_key)

    def add_lr_scheduler_args(self, cls, link_to: str = "model.scheduler_init", nested_key: str = "lr_scheduler"):
        self.lr_scheduler = (cls, link_to, nested_key)

    def add_class_arguments(self, cls, nested_key: str, **_):
        self.class_args[nested_key] = cls

    def add_argument(self, name: str, default=None, **_):
        self.extra_args[name.lstrip("-")] = default


class CLI:
    """Base CLI; task scripts override :meth:`add_arguments_to_parser` like LightningCLI."""

    # like the reference: scripts/trainer.yaml relative to the working directory, falling
    # back to the copy shipped in the package
    trainer_defaults_file = os.path.join("scripts", "trainer.yaml")
    package_defaults_file = os.path.join(os.path.dirname(os.path.abspath(__file__)), "trainer.yaml")

    def __init__(self, model_class, description: str = "", run: bool = True, args: Optional[List[str]] = None,
                 save_config: bool = True, **_):
        self.model_class = model_class
        self.description = description
        self.parser = CLIParser()
        self.add_default_arguments_to_parser(self.parser)
        self.add_arguments_to_parser(self.parser)
        argv = list(sys.argv[1:] if args is None else args)
        self.subcommand, self.config = self.parse(argv)
        self.save_config = save_config
        if self.config.pop("print_config", False):
            print(yaml.safe_dump(self.config, sort_keys=False))
            sys.exit(0)
        self._maybe_launch(argv)
        self.instantiate()
        if run and self.subcommand:
            getattr(self, f"run_{self.subcommand}")()

    # -- LightningCLI hooks ----------------------------------------------------------------
    def add_default_arguments_to_parser(self, parser: CLIParser):
        parser.add_argument("--experiment", default="default")

    def add_arguments_to_parser(self, parser: CLIParser):
        from ..train.loggers import TensorBoardLogger

        parser.add_class_arguments(TensorBoardLogger, "logger")
        parser.link_arguments("trainer.default_root_dir", "logger.save_dir", apply_on="parse")
        parser.link_arguments("experiment", "logger.name", apply_on="parse")
        import torch

        parser.add_optimizer_args(torch.optim.AdamW, link_to="model.optimizer_init")

    # -- parsing ------------------------------------------------------------------------------
    def _base_config(self) -> Dict[str, Any]:
        cfg: Dict[str, Any] = {"model": {}, "data": {}, "trainer": {}}
        for k, v in self.parser.extra_args.items():
            cfg[k] = v
        if self.parser.optimizer:
            cls, _, key = self.parser.optimizer
            cfg[key] = _signature_defaults(cls, skip=("self", "params"))
        if self.parser.lr_scheduler:
            cls, _, key = self.parser.lr_scheduler
            cfg[key] = _signature_defaults(cls, skip=("self", "optimizer"))
        for key, cls in self.parser.class_args.items():
            cfg[key] = _signature_defaults(cls)
        return cfg

    def parse(self, argv: List[str]):
        sub = None
        if argv and argv[0] in SUBCOMMANDS:
            sub, argv = argv[0], argv[1:]
        elif argv and not argv[0].startswith("-"):
            raise SystemExit(f"unknown subcommand {argv[0]!r}; expected one of {SUBCOMMANDS}")
        cfg = self._base_config()
        dfile = self.trainer_defaults_file if os.path.exists(self.trainer_defaults_file) else self.package_defaults_file
        if os.path.exists(dfile):
            with open(dfile) as f:
                _merge(cfg, yaml.safe_load(f) or {})
        for k, v in self.parser.defaults.items():
            _set(cfg, k, copy.deepcopy(v))
        # pairs "--a.b=v" or "--a.b v"
        pairs = []
        i = 0
        while i < len(argv):
            a = argv[i]
            if not a.startswith("--"):
                raise SystemExit(f"unexpected argument {a!r}")
            if "=" in a:
                k, v = a[2:].split("=", 1)
            elif a[2:] in ("print_config",):
                k, v = a[2:], "true"
            else:
                k = a[2:]
                i += 1
                if i >= len(argv):
                    raise SystemExit(f"missing value for {a}")
                v = argv[i]
            pairs.append((k, v))
            i += 1
        for k, v in pairs:
            if k == "config":
                with open(v) as f:
                    _merge(cfg, yaml.safe_load(f) or {})
        for k, v in pairs:
            if k == "config":
                continue
            val = _parse_value(v)
            if k == "data" and isinstance(val, str):
                cfg.setdefault("data", {})
                if not isinstance(cfg["data"], dict):
                    cfg["data"] = {}
                cfg["data"]["class"] = val
            else:
                _set(cfg, k, val)
        for src, dst, fn, when in self.parser.links:
            if when == "parse":
                val = _get(cfg, src)
                if val is not None:
                    _set(cfg, dst, fn(val) if fn else val)
        return sub, cfg

    # -- instantiation ------------------------------------------------------------------------
    def _devices(self) -> int:
        from ..train.trainer import Trainer

        t = self.config.get("trainer", {})
        acc = str(t.get("accelerator") or "auto").lower()
        if acc not in ("gpu", "cuda", "auto"):
            return 1
        from ..parallel.launch import gpu_count

        if gpu_count() == 0:  # counted without initialising HIP in this (launcher) process
            return 1
        return Trainer._parse_devices(t.get("devices") if t.get("devices") is not None else t.get("gpus"))

    def _maybe_launch(self, argv):
        n = self._devices()
        if n > 1 and "WORLD_SIZE" not in os.environ:
            from ..parallel.launch import spawn

            sys.exit(spawn(n, [sys.executable, sys.argv[0]] + argv))

    def instantiate(self):
        from ..data.registry import DATAMODULE_REGISTRY
        from ..train.module import import_class
        from ..train.trainer import Trainer

        cfg = self.config
        seed = cfg.get("seed_everything")
        if seed is not None:
            import torch

            torch.manual_seed(int(seed))
        data = dict(cfg.get("data") or {})
        dm_name = data.pop("class", None) or data.pop("class_path", None)
        self.datamodule = None
        if dm_name:
            dm_cls = DATAMODULE_REGISTRY.get(dm_name.split(".")[-1])
            if dm_cls is None:
                raise SystemExit(f"unknown data module {dm_name!r}; registered: {sorted(DATAMODULE_REGISTRY)}")
            self.datamodule = dm_cls(**data)
        model_cfg = dict(cfg.get("model") or {})
        for src, dst, fn, when in self.parser.links:
            if when == "instantiate" and src.startswith("data.") and self.datamodule is not None:
                val = getattr(self.datamodule, src.split(".", 1)[1])
                if isinstance(val, tuple):
                    val = list(val)
                _set(cfg, dst, fn(val) if fn else val)
                if dst.startswith("model."):
                    model_cfg[dst.split(".", 1)[1]] = val
        if self.parser.optimizer:
            ocls, link, key = self.parser.optimizer
            model_cfg[link.split(".", 1)[1]] = {"class_path": f"{ocls.__module__}.{ocls.__name__}".replace(
                "torch.optim.adamw", "torch.optim"), "init_args": dict(cfg.get(key) or {})}
        if self.parser.lr_scheduler:
            scls, link, key = self.parser.lr_scheduler
            model_cfg[link.split(".", 1)[1]] = {"class_path": f"torch.optim.lr_scheduler.{scls.__name__}",
                                                "init_args": dict(cfg.get(key) or {})}
        self.model = self.model_class(**model_cfg)
        tcfg = dict(cfg.get("trainer") or {})
        callbacks = []
        for cb in tcfg.pop("callbacks", None) or []:
            if isinstance(cb, dict) and "class_path" in cb:
                callbacks.append(import_class(cb["class_path"])(**(cb.get("init_args") or {})))
        logger_flag = tcfg.pop("logger", True)
        logger = None
        if logger_flag:
            lcfg = dict(cfg.get("logger") or {})
            from ..train.loggers import TensorBoardLogger

            lcfg.setdefault("save_dir", tcfg.get("default_root_dir") or "logs")
            logger = TensorBoardLogger(**{k: v for k, v in lcfg.items() if v is not None or k == "version"})
        self.trainer = Trainer(logger=logger if logger is not None else False, callbacks=callbacks, **tcfg)
        if self.save_config and logger is not None and self.trainer.is_global_zero and self.subcommand:
            os.makedirs(logger.log_dir, exist_ok=True)
            with open(os.path.join(logger.log_dir, "config.yaml"), "w") as f:
                yaml.safe_dump(_jsonable(cfg), f, sort_keys=False)

    # -- subcommands ---------------------------------------------------------------------------
    def run_fit(self):
        self.trainer.fit(self.model, datamodule=self.datamodule)

    def run_validate(self):
        self.trainer.validate(self.model, datamodule=self.datamodule)

    def run_test(self):
        self.trainer.test(self.model, datamodule=self.datamodule)


def _jsonable(o):
    if isinstance(o, dict):
        return {str(k): _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, (str, int, float, bool)) or o is None:
        return o
    return str(o)


def freeze(module):
    from ..utils.misc import freeze as _f

    _f(module)
