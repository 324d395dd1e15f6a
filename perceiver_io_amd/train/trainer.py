"""A lean Trainer with the PyTorch-Lightning 1.5 surface the reference uses.

Reference call stack: SURVEY §3.2 (``Trainer.fit`` under DDP) — prepare_data on rank 0 →
setup → configure_optimizers → parameter broadcast → sanity validation → epochs of
(train step, log, optimizer, per-step scheduler) → validation epoch → ModelCheckpoint.
Flags mirror ``scripts/trainer.yaml`` (max_steps / max_epochs, limit_*_batches,
val_check_interval, check_val_every_n_epoch, log_every_n_steps, num_sanity_val_steps,
accumulate_grad_batches, gradient_clip_val, precision, resume_from_checkpoint,
fast_dev_run, overfit_batches, terminate_on_nan, detect_anomaly, deterministic, profiler).

MI355X specifics:
  * ``precision`` ``bf16`` (default in this framework's trainer.yaml) runs the fused HIP
    kernels (bf16 MFMA, fp32 master weights / optimizer); ``32`` runs the eager fp32 path
    (the reference's exact numerics) — both on the GPU.
  * AdamW from ``configure_optimizers`` is swapped for ``FusedAdamW`` over a flat parameter
    buffer (same hyper-parameters and state-dict layout), and the step is captured once in a
    hipGraph and replayed (``graph_capture``), per batch shape.
  * multi-GPU: one process per GPU (``devices``), RCCL process group, flat-buffer gradient
    all-reduce (``parallel/reducer.py``), rank-sharded samplers.
"""
from __future__ import annotations

import contextlib
import math
import os
import sys
import time
import warnings
from typing import Any, Dict, List, Optional

import torch

from .. import ops
from ..parallel import dist as pdist
from .callbacks import Callback, LearningRateMonitor, ModelCheckpoint
from .checkpoint import load_checkpoint, make_checkpoint, save_checkpoint
from .engine import StepEngine, _to
from .loggers import TensorBoardLogger


def _as_limit(v, n: int) -> int:
    if v is None:
        return n
    if isinstance(v, float) and v <= 1.0:
        return int(math.ceil(n * v)) if v > 0 else 0
    return min(n, int(v))


class _Timer:
    def __init__(self):
        self.t: Dict[str, float] = {}
        self.n: Dict[str, int] = {}

    @contextlib.contextmanager
    def __call__(self, name):
        t0 = time.perf_counter()
        yield
        self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0
        self.n[name] = self.n.get(name, 0) + 1

    def summary(self) -> str:
        rows = [f"{k:28s} {self.n[k]:8d} {self.t[k]:10.3f}s {1e3 * self.t[k] / max(1, self.n[k]):9.3f}ms"
                for k in sorted(self.t, key=lambda k: -self.t[k])]
        return "\n".join(["action                          calls      total      mean"] + rows)


class _TorchProfiler:
    """``--trainer.profiler=pytorch``: torch.profiler (ROCm activity tracing) over training steps
    ``wait``..``wait+active``; writes a Chrome trace and a per-kernel table into
    ``<log_dir>/profiler/``.  ``advanced`` also records shapes and stacks."""

    def __init__(self, out_dir: str, advanced: bool = False, wait: int = 3, active: int = 5):
        from torch.profiler import ProfilerActivity, profile, schedule

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
        self.out_dir = out_dir
        self.prof = profile(activities=acts, schedule=schedule(wait=wait, warmup=1, active=active, repeat=1),
                            record_shapes=advanced, with_stack=advanced, on_trace_ready=self._ready)
        self.prof.__enter__()
        self.done = False

    def _ready(self, prof):
        os.makedirs(self.out_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(self.out_dir, "trace.json"))
        key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
        with open(os.path.join(self.out_dir, "kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by=key, row_limit=60))
        self.done = True

    def step(self):
        if not self.done:
            self.prof.step()

    def close(self):
        self.prof.__exit__(None, None, None)


class Trainer:
    def __init__(self, logger: Any = True, checkpoint_callback: Optional[bool] = None, enable_checkpointing: bool = True,
                 callbacks: Optional[List[Callback]] = None, default_root_dir: Optional[str] = None,
                 gradient_clip_val: Optional[float] = None, gradient_clip_algorithm: Optional[str] = None,
                 num_nodes: int = 1, num_processes: int = 1, devices: Any = None, gpus: Any = None,
                 accelerator: Optional[str] = None, strategy: Optional[str] = None, enable_progress_bar: bool = True,
                 overfit_batches: float = 0.0, check_val_every_n_epoch: int = 1, fast_dev_run: Any = False,
                 accumulate_grad_batches: Optional[int] = None, max_epochs: Optional[int] = None,
                 min_epochs: Optional[int] = None, max_steps: int = -1, min_steps: Optional[int] = None,
                 max_time: Any = None, limit_train_batches: Any = 1.0, limit_val_batches: Any = 1.0,
                 limit_test_batches: Any = 1.0, limit_predict_batches: Any = 1.0, val_check_interval: Any = 1.0,
                 log_every_n_steps: int = 50, precision: Any = "bf16", num_sanity_val_steps: int = 2,
                 resume_from_checkpoint: Optional[str] = None, profiler: Optional[str] = None, benchmark: bool = False,
                 deterministic: bool = False, detect_anomaly: bool = False, terminate_on_nan: Optional[bool] = None,
                 replace_sampler_ddp: bool = True, graph_capture: Optional[bool] = None, seed: Optional[int] = None,
                 allreduce_dtype: Optional[str] = None, **ignored: Any):
        for k, v in ignored.items():
            if v not in (None, False, 0, 0.0, "", [], {}) and k not in _KNOWN_NOOP:
                warnings.warn(f"Trainer flag {k}={v!r} has no effect in this framework")
        self.default_root_dir = default_root_dir or os.getcwd()
        self.callbacks: List[Callback] = list(callbacks or [])
        self.enable_checkpointing = enable_checkpointing and checkpoint_callback is not False
        if self.enable_checkpointing and not any(isinstance(c, ModelCheckpoint) for c in self.callbacks):
            self.callbacks.append(ModelCheckpoint())
        if not self.enable_checkpointing:
            self.callbacks = [c for c in self.callbacks if not isinstance(c, ModelCheckpoint)]
        self.gradient_clip_val = gradient_clip_val or 0.0
        self.max_epochs = max_epochs
        self.max_steps = max_steps if max_steps is not None else -1
        self.min_steps = min_steps
        self.limit_train_batches = limit_train_batches
        self.limit_val_batches = limit_val_batches
        self.limit_test_batches = limit_test_batches
        self.val_check_interval = val_check_interval
        self.check_val_every_n_epoch = check_val_every_n_epoch or 1
        self.log_every_n_steps = max(1, int(log_every_n_steps))
        self.precision = str(precision)
        self.num_sanity_val_steps = num_sanity_val_steps
        self.resume_from_checkpoint = resume_from_checkpoint
        self.accumulate = int(accumulate_grad_batches or 1)
        self.enable_progress_bar = enable_progress_bar
        self.overfit_batches = overfit_batches
        self.terminate_on_nan = bool(terminate_on_nan)
        self.profiler_name = profiler
        self.timer = _Timer()
        self.deterministic = deterministic
        self.detect_anomaly = detect_anomaly
        self.replace_sampler_ddp = replace_sampler_ddp
        self.graph_capture = graph_capture
        self.seed = seed
        # gradient all-reduce wire format (SURVEY C-03): None / "fp32" (parity default) or "bf16"
        # (half the bytes over xGMI; every rank still applies the same reduced gradient)
        if allreduce_dtype not in (None, "fp32", "float32", "bf16", "bfloat16"):
            raise ValueError(f"allreduce_dtype must be fp32 or bf16, got {allreduce_dtype!r}")
        self.allreduce_dtype = torch.bfloat16 if allreduce_dtype in ("bf16", "bfloat16") else None
        if fast_dev_run:
            n = 1 if fast_dev_run is True else int(fast_dev_run)
            self.limit_train_batches = self.limit_val_batches = self.limit_test_batches = n
            self.max_steps, self.max_epochs, self.num_sanity_val_steps = n, 1, 0
            logger = False
        self.fast_dev_run = bool(fast_dev_run)
        # devices / accelerator
        self.accelerator = (accelerator or ("gpu" if gpus else None) or "auto").lower()
        want_gpu = self.accelerator in ("gpu", "cuda", "auto") and torch.cuda.is_available()
        if self.accelerator in ("gpu", "cuda") and not torch.cuda.is_available():
            warnings.warn("accelerator=gpu requested but no GPU is visible; running on CPU")
        self.on_gpu = want_gpu
        self.requested_devices = self._parse_devices(devices if devices is not None else gpus)
        self.dist = pdist.init(device_type="cuda" if self.on_gpu else "cpu")
        self.device = (torch.device("cuda", torch.cuda.current_device()) if self.on_gpu else torch.device("cpu"))
        # logger
        if logger is True:
            self.logger = TensorBoardLogger(save_dir=self.default_root_dir, name="default")
        elif logger is False or logger is None:
            self.logger = None
        else:
            self.logger = logger
        if self.logger is not None and not self.dist.is_main:
            self.logger = None if not isinstance(self.logger, TensorBoardLogger) else _NullLogger(self.logger)
        # state
        self.global_step = 0
        self.current_epoch = 0
        self.should_stop = False
        self.sanity_checking = False
        self.callback_metrics: Dict[str, float] = {}
        self.logged_metrics: Dict[str, float] = {}
        self.progress_bar_metrics: Dict[str, float] = {}
        self._step_logs: Dict[str, Any] = {}
        self._epoch_logs: Dict[str, List] = {}
        self.optimizers: List[Any] = []
        self.lr_schedulers: List[Any] = []
        self.datamodule = None
        self.model = None
        self._engine: Optional[StepEngine] = None

    @staticmethod
    def _parse_devices(d) -> int:
        from ..parallel.launch import gpu_count as _gpu_count  # no HIP init (launcher parent)

        if d is None:
            return 1
        if isinstance(d, str):
            d = d.strip()
            if d in ("-1", "auto"):
                return max(1, _gpu_count())
            if "," in d:
                return len([x for x in d.split(",") if x.strip()])
            d = int(d)
        if isinstance(d, (list, tuple)):
            return len(d)
        d = int(d)
        return max(1, _gpu_count()) if d == -1 else max(1, d)

    # ------------------------------------------------------------------------------------
    @property
    def is_global_zero(self) -> bool:
        return self.dist.is_main

    def is_global_zero_or_all(self) -> bool:
        return True  # every rank tracks callback state; only rank 0 writes files

    @property
    def world_size(self) -> int:
        return self.dist.world_size

    def _backend_ctx(self):
        if not self.on_gpu:
            return ops.backend("torch") if ops.get_backend() == "auto" else contextlib.nullcontext()
        if self.precision in ("32", "32-true", "64"):
            return ops.backend("torch")
        return contextlib.nullcontext()

    @property
    def fused(self) -> bool:
        return self.on_gpu and self.precision not in ("32", "32-true", "64") and ops.get_backend() in ("auto", "hip")

    # ---- logging ------------------------------------------------------------------------
    def _log(self, name, value, prog_bar=False, on_step=None, on_epoch=None, sync_dist=False):
        if self.sanity_checking:
            return
        if self._in_train:
            self._step_logs[name] = value
            if prog_bar:
                self.progress_bar_metrics[name] = value
        else:
            self._epoch_logs.setdefault(name, []).append((value, self._cur_bs))

    def log_scalars(self, metrics: Dict[str, float]):
        if self.logger is not None:
            self.logger.log_metrics({k: float(v) for k, v in metrics.items()}, self.global_step)

    # ---- setup --------------------------------------------------------------------------
    def _configure_optimizers(self, model):
        res = model.configure_optimizers()
        sched = None
        if isinstance(res, dict):
            opt = res["optimizer"]
            ls = res.get("lr_scheduler")
            sched = ls["scheduler"] if isinstance(ls, dict) else ls
        elif isinstance(res, (list, tuple)):
            opt = res[0][0] if isinstance(res[0], (list, tuple)) else res[0]
            if len(res) > 1:
                s = res[1][0] if isinstance(res[1], (list, tuple)) else res[1]
                sched = s["scheduler"] if isinstance(s, dict) else s
        else:
            opt = res
        if self.fused and type(opt).__name__ in ("AdamW", "Adam"):
            from ..ops.optim import FusedAdamW

            g = opt.param_groups[0]
            wd = g.get("weight_decay", 0.0)
            if type(opt).__name__ == "Adam" and wd:
                warnings.warn("Adam with L2 weight decay is executed as decoupled AdamW by the fused optimizer")
            new = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=g["lr"], betas=g["betas"],
                             eps=g["eps"], weight_decay=wd, max_grad_norm=self.gradient_clip_val)
            if sched is not None:
                init = getattr(model.hparams, "get", lambda *_: None)("scheduler_init")
                if init is not None:
                    from .module import instantiate_class

                    sched = instantiate_class(new, init)
                else:
                    warnings.warn("scheduler could not be re-bound to the fused optimizer; dropped")
                    sched = None
            opt = new
        return opt, sched

    def _attach(self, model, datamodule):
        self.model = model
        model._trainer = self
        self.datamodule = datamodule
        model.to(self.device)

    def _loader(self, dl, shuffle: bool):
        if dl is None:
            return None
        if self.world_size > 1 and self.replace_sampler_ddp and isinstance(dl, torch.utils.data.DataLoader):
            from ..parallel.sampler import ShardedSampler

            samp = ShardedSampler(len(dl.dataset), self.dist.rank, self.world_size, shuffle=shuffle)
            dl = torch.utils.data.DataLoader(dl.dataset, batch_size=dl.batch_size, sampler=samp,
                                             collate_fn=dl.collate_fn, num_workers=dl.num_workers,
                                             pin_memory=dl.pin_memory, drop_last=dl.drop_last)
        return dl

    # ---- public API -----------------------------------------------------------------------
    def fit(self, model, datamodule=None, train_dataloaders=None, val_dataloaders=None, ckpt_path=None):
        if self.seed is not None:
            torch.manual_seed(self.seed + self.dist.rank)
        if self.deterministic:  # atomics-free kernel reductions + torch's deterministic algorithms
            torch.use_deterministic_algorithms(True, warn_only=True)
            ops.set_deterministic(True)
        torch.autograd.set_detect_anomaly(self.detect_anomaly)
        if datamodule is not None:
            if self.dist.local_rank == 0:
                datamodule.prepare_data()
            pdist.barrier()
            datamodule.setup("fit")
            train_dataloaders = train_dataloaders or datamodule.train_dataloader()
            if val_dataloaders is None and hasattr(datamodule, "val_dataloader"):
                val_dataloaders = datamodule.val_dataloader()
        self._attach(model, datamodule)
        train_dl = self._loader(train_dataloaders, True)
        val_dl = self._loader(val_dataloaders, False)
        with self._backend_ctx():
            opt, sched = self._configure_optimizers(model)
            self.optimizers = [opt]
            self.lr_schedulers = [sched] if sched is not None else []
            reducer = None
            if self.world_size > 1:
                from ..ops.optim import FlatParameterSpace
                from ..parallel.reducer import FlatGradReducer

                flat = getattr(opt, "flat", None) or FlatParameterSpace(
                    [p for p in model.parameters() if p.requires_grad], with_shadow=False)
                reducer = FlatGradReducer(flat, wire_dtype=self.allreduce_dtype)
                net = getattr(model, "model", None)
                if net is not None:  # ready points: decoder + head, then layer_n (overlapped all-reduce)
                    reducer.plan(net)
                reducer.broadcast_parameters(model)
            if not self.fused and self.gradient_clip_val:
                warnings.warn("gradient clipping on the eager path uses torch.nn.utils.clip_grad_norm_")
            ckpt_path = ckpt_path or self.resume_from_checkpoint
            if ckpt_path:
                self._restore(ckpt_path)
            use_graph = self.graph_capture if self.graph_capture is not None else self.fused
            # the metric tensors a captured step logs are static outputs of THAT graph: saved per
            # graph, restored before its replays
            hooks = (lambda: dict(self._step_logs), self._restore_step_logs)
            self._engine = StepEngine(self._training_loss, opt, sched, reducer=reducer, device=self.device,
                                      graph=bool(use_graph), accumulate=self.accumulate, state_hooks=hooks)
            if self.logger is not None and self.is_global_zero:
                self.logger.log_hyperparams(dict(model.hparams))
            for cb in self.callbacks:
                cb.on_fit_start(self, model)
            if val_dl is not None and self.num_sanity_val_steps:
                self.sanity_checking = True
                self._run_eval(val_dl, "validation", limit=self.num_sanity_val_steps)
                self.sanity_checking = False
            try:
                self._fit_loop(train_dl, val_dl)
            finally:
                if reducer is not None:
                    reducer.close()  # never the target of a later fit's ready points
            for cb in self.callbacks:
                cb.on_fit_end(self, model)
        if self.logger is not None:
            self.logger.finalize()
        if self.profiler_name and self.is_global_zero:
            print(self.timer.summary(), file=sys.stderr)
        return self

    def validate(self, model=None, datamodule=None, dataloaders=None, ckpt_path=None, verbose: bool = True):
        return self._eval_entry(model, datamodule, dataloaders, ckpt_path, "validation", verbose)

    def test(self, model=None, datamodule=None, dataloaders=None, ckpt_path=None, verbose: bool = True):
        return self._eval_entry(model, datamodule, dataloaders, ckpt_path, "test", verbose)

    def _eval_entry(self, model, datamodule, dataloaders, ckpt_path, stage, verbose):
        model = model or self.model
        if datamodule is not None:
            if self.dist.local_rank == 0:
                datamodule.prepare_data()
            pdist.barrier()
            datamodule.setup(stage if stage == "test" else "validate")
            dataloaders = dataloaders or (datamodule.test_dataloader() if stage == "test" else datamodule.val_dataloader())
        self._attach(model, datamodule)
        if ckpt_path:
            sd = load_checkpoint(ckpt_path)["state_dict"]
            model.load_state_dict(sd)
        with self._backend_ctx():
            res = self._run_eval(self._loader(dataloaders, False), stage)
        if verbose and self.is_global_zero:
            print({k: round(v, 5) for k, v in res.items()}, file=sys.stderr)
        return [res]

    # ---- loops ---------------------------------------------------------------------------
    _in_train = False
    _cur_bs = 1

    def _restore_step_logs(self, logs):
        self._step_logs = dict(logs)
        for k in self.progress_bar_metrics:
            if k in logs:
                self.progress_bar_metrics[k] = logs[k]

    def _training_loss(self, batch):
        out = self.model.training_step(batch, self._batch_idx)
        return out["loss"] if isinstance(out, dict) else out

    def _fit_loop(self, train_dl, val_dl):
        model = self.model
        n_train = len(train_dl)
        if self.overfit_batches:
            n_train = _as_limit(self.overfit_batches, n_train)
        n_train = _as_limit(self.limit_train_batches, n_train)
        vci = self.val_check_interval
        val_every = n_train if (isinstance(vci, float) and vci >= 1.0) else (
            max(1, int(n_train * vci)) if isinstance(vci, float) else int(vci))
        max_epochs = self.max_epochs if self.max_epochs is not None else (1000 if self.max_steps < 0 else 10 ** 9)
        t_last, steps_last = time.perf_counter(), self.global_step
        tprof = None
        if self.profiler_name in ("pytorch", "advanced") and self.is_global_zero:
            base = self.logger.log_dir if self.logger is not None else (self.default_root_dir or ".")
            tprof = _TorchProfiler(os.path.join(base, "profiler"), advanced=self.profiler_name == "advanced")
        while self.current_epoch < max_epochs and not self.should_stop:
            model.train()
            sampler = getattr(train_dl, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(self.current_epoch)
            acc_buf = []
            for bi, batch in enumerate(train_dl):
                if bi >= n_train or self.should_stop:
                    break
                self._batch_idx = bi
                self._in_train = True
                batch = _to(batch, self.device)
                if self._engine.graph_enabled:
                    batch = model.graph_batch(batch)  # bounded set of shapes → bounded set of graphs
                acc_buf.append(batch)
                if len(acc_buf) < self.accumulate:
                    continue
                with self.timer("training_step_and_update"):
                    if not self.fused and self.gradient_clip_val:
                        loss = self._eager_clip_step(acc_buf)
                    else:
                        loss = self._engine.step(acc_buf if self.accumulate > 1 else acc_buf[0], ring_view=True)
                acc_buf = []
                self._in_train = False
                self.global_step += 1
                if tprof is not None:
                    tprof.step()
                for cb in self.callbacks:
                    cb.on_train_batch_end(self, model)
                if self.global_step % self.log_every_n_steps == 0 or self.fast_dev_run:
                    vals = {k: float(v.detach().float().item() if torch.is_tensor(v) else v)
                            for k, v in self._step_logs.items()}
                    now = time.perf_counter()
                    sps = (self.global_step - steps_last) / max(now - t_last, 1e-9)
                    t_last, steps_last = now, self.global_step
                    vals["steps_per_sec"] = sps
                    self.callback_metrics.update(vals)
                    self.log_scalars(vals)
                    ops.mlm_head.check_overflow()  # fixed-capacity MLM rows: fail loudly, never truncate
                    ops.check_device_errors()  # persistent-kernel spin timeouts, checked-build index errors
                    if self.terminate_on_nan and not all(math.isfinite(v) for v in vals.values()):
                        raise ValueError(f"non-finite metric at step {self.global_step}: {vals}")
                    if self.enable_progress_bar and self.is_global_zero:
                        pb = " ".join(f"{k}={v:.4g}" for k, v in vals.items())
                        print(f"epoch {self.current_epoch} step {self.global_step} {pb}", file=sys.stderr, flush=True)
                if 0 < self.max_steps <= self.global_step:
                    self.should_stop = True
                if val_dl is not None and (bi + 1) % val_every == 0 and \
                        (self.current_epoch + 1) % self.check_val_every_n_epoch == 0:
                    self._run_eval(val_dl, "validation")
                    model.train()
            for cb in self.callbacks:
                cb.on_train_epoch_end(self, model)
            self.current_epoch += 1
        if tprof is not None:
            tprof.close()
        ops.check_device_errors()

    def _eager_clip_step(self, batches):
        opt = self.optimizers[0]
        red = self._engine.reducer
        for i, b in enumerate(batches):
            if red is not None and red.enabled:  # ready points only in the last micro-batch's backward
                red.arm() if i == len(batches) - 1 else red.disarm()
            loss = self._training_loss(b)
            (loss / len(batches)).backward()
        if red is not None:
            red.finish()
            if red.enabled:  # all-reduced SUM → mean before clipping (clip the mean's norm)
                for p in self.model.parameters():
                    if p.grad is not None:
                        p.grad.mul_(red.grad_scale())
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.gradient_clip_val)
        opt.step()
        for s in self.lr_schedulers:
            s.step()
        if self._engine.reducer is not None:
            self._engine.reducer.flat.zero_grad()
        else:
            opt.zero_grad()
        return loss.detach()

    @torch.no_grad()
    def _run_eval(self, dl, stage: str, limit: Optional[int] = None) -> Dict[str, float]:
        if dl is None:
            return {}
        model = self.model
        was = model.training
        model.eval()
        self._epoch_logs = {}
        n = len(dl)
        lim = _as_limit(self.limit_val_batches if stage == "validation" else self.limit_test_batches, n)
        if limit is not None:
            lim = min(lim, limit)
        step_fn = model.validation_step if stage == "validation" else model.test_step
        with self.timer(f"{stage}_loop"):
            for bi, batch in enumerate(dl):
                if bi >= lim:
                    break
                batch = _to(batch, self.device)
                bs = _batch_size(batch)
                self._cur_bs = bs
                step_fn(batch, bi)
        res = {}
        for k, vals in self._epoch_logs.items():
            tot = sum(w for _, w in vals)
            res[k] = sum(float(v.detach().float().item() if torch.is_tensor(v) else v) * w for v, w in vals) / max(tot, 1)
        if self.world_size > 1:
            res = {k: pdist.all_reduce_mean(v) for k, v in res.items()}
        if not self.sanity_checking:
            self.callback_metrics.update(res)
            self.log_scalars(res)
            if stage == "validation":
                model.on_validation_epoch_end()
                for cb in self.callbacks:
                    cb.on_validation_end(self, model)
        model.train(was)
        return res

    # ---- checkpointing -------------------------------------------------------------------
    def save_checkpoint(self, path: str):
        cbs = {cb.state_key(): cb.state_dict() for cb in self.callbacks if cb.state_dict()}
        ckpt = make_checkpoint(self.model, self.current_epoch, self.global_step, self.optimizers, self.lr_schedulers, cbs)
        if self.is_global_zero:
            save_checkpoint(ckpt, path)
        pdist.barrier()

    def _restore(self, path: str):
        ckpt = load_checkpoint(path)
        self.model.load_state_dict(ckpt["state_dict"])
        for o, s in zip(self.optimizers, ckpt.get("optimizer_states", [])):
            o.load_state_dict(s)
        for sc, s in zip(self.lr_schedulers, ckpt.get("lr_schedulers", [])):
            sc.load_state_dict(s)
        self.global_step = int(ckpt.get("global_step", 0))
        self.current_epoch = int(ckpt.get("epoch", 0)) + 1
        for cb in self.callbacks:
            st = ckpt.get("callbacks", {}).get(cb.state_key())
            if st:
                cb.load_state_dict(st)


_KNOWN_NOOP = {"process_position", "auto_select_gpus", "tpu_cores", "ipus", "log_gpu_memory",
               "progress_bar_refresh_rate", "track_grad_norm", "flush_logs_every_n_steps", "sync_batchnorm",
               "enable_model_summary", "weights_summary", "weights_save_path", "reload_dataloaders_every_n_epochs",
               "reload_dataloaders_every_epoch", "auto_lr_find", "auto_scale_batch_size", "prepare_data_per_node",
               "plugins", "amp_backend", "amp_level", "move_metrics_to_cpu", "multiple_trainloader_mode",
               "stochastic_weight_avg", "limit_predict_batches", "min_epochs", "max_time"}


def _batch_size(batch) -> int:
    if torch.is_tensor(batch):
        return batch.shape[0] if batch.dim() else 1
    if isinstance(batch, (list, tuple)):
        for b in batch:
            if torch.is_tensor(b) and b.dim():
                return b.shape[0]
    return 1


class _NullLogger:
    """Non-zero ranks: same attributes (log_dir for checkpoint paths), writes nothing."""

    def __init__(self, base):
        self._base = base

    @property
    def log_dir(self):
        return self._base.log_dir

    def log_metrics(self, *a, **k): ...
    def log_hyperparams(self, *a, **k): ...
    def add_text(self, *a, **k): ...
    def add_scalar(self, *a, **k): ...
    def finalize(self, *a, **k): ...
