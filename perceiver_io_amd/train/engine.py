"""Training-step engine: forward+backward → gradient all-reduce → fused optimizer, with
optional hipGraph capture of the whole step.

The Perceiver step is launch/latency-bound on MI355X (the reference issues
~2,000 kernels per step for a few hundred GFLOP), so instead of a tracing compiler the
engine captures the step once into a hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on
ROCm) and replays it: one host call per step, no per-kernel launch overhead, no Python in
the loop.  Everything inside the step is capture-safe by construction: no host syncs
(sync-free masking, fixed-capacity MLM row compaction); masking draws from its own device
counter-hash state (``ops/masking.py``) and dropout seeds from torch's graph-aware generator,
both advanced on every replay; optimizer hyper-parameters are read from device memory (staged
before replay).

Gradient accumulation: ``accumulate`` micro-batches per optimizer step (the all-reduce and
update run only on the last one, as in Lightning's ``accumulate_grad_batches``) — on the graph
path as ``accumulate - 1`` "micro" graph replays plus one "last" graph.

Variable batch shapes (the reference's IMDB collator pads to the longest sequence of each
batch, ``data/imdb.py:52-63``, and its loaders keep the partial last batch): captured graphs
are cached per batch *shape signature* (tensor shapes + dtypes), at most ``max_graphs`` of
them (least recently used evicted, each with its own private memory pool so an evicted
graph's memory is really released).  Task modules bucket text lengths before the step
(``LitModuleBase.graph_batch``: pad to a multiple of 64, pad keys masked — identical
semantics), so an epoch of pad-to-longest batches needs a handful of graphs, not hundreds.
"""
from __future__ import annotations

import os
import random

from collections import OrderedDict
from typing import Callable, Dict, Optional

import torch


def _copy_into(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_into(d, s)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])


def _pairs(dst, src, out):
    if isinstance(dst, torch.Tensor):
        out.append((dst, src))
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _pairs(d, s, out)
    elif isinstance(dst, dict):
        for k in dst:
            _pairs(dst[k], src[k], out)
    return out


def _stage_step(dst, src, opt=None, seeds=None) -> None:
    """Copy a batch into a captured graph's static buffers and (``opt``) stage the optimizer's
    per-step hyper-parameters and (``seeds`` = (pool, values)) the graph's dropout seeds, in ONE
    kernel launch (``stage_step``) for the device-resident tensors; host tensors or odd layouts
    take ``copy_``."""
    from ..ops import ext

    pairs = _pairs(dst, src, [])
    fast, slow = [], []
    for d, s in pairs:
        ok = (isinstance(s, torch.Tensor) and s.device == d.device and s.dtype == d.dtype and s.numel() == d.numel()
              and s.is_contiguous() and d.is_contiguous())
        (fast if ok and len(fast) < 8 else slow).append((d, s))
    for d, s in slow:
        d.copy_(s, non_blocking=True)
    hyper = opt is not None and opt.hyper.is_cuda
    if fast or hyper or seeds is not None:
        ext.require().stage_step([d for d, _ in fast], [s for _, s in fast], opt.hyper if hyper else None,
                                 opt.hyper_values() if hyper else [],
                                 seed_dst=seeds[0] if seeds is not None else None,
                                 seeds=seeds[1] if seeds is not None else [])
    if opt is not None and not hyper:
        opt.stage_hyper()


def _clone_to(obj, device):
    if isinstance(obj, torch.Tensor):
        return obj.to(device, non_blocking=True).clone()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_clone_to(o, device) for o in obj)
    if isinstance(obj, dict):
        return {k: _clone_to(v, device) for k, v in obj.items()}
    return obj


def shape_key(obj):
    """Hashable signature of a (nested) batch: tensor shapes/dtypes, other leaves by value."""
    if isinstance(obj, torch.Tensor):
        return ("T", tuple(obj.shape), obj.dtype)
    if isinstance(obj, (list, tuple)):
        return (type(obj).__name__,) + tuple(shape_key(o) for o in obj)
    if isinstance(obj, dict):
        return ("D",) + tuple((k, shape_key(obj[k])) for k in sorted(obj))
    return ("V", obj)


# replayed steps return their loss as a slot of a device ring written by the captured update
# kernel: a returned loss stays valid for this many steps (no per-step copy launch)
LOSS_RING = 1024


class _Captured:
    """One captured step: the graph, its static input batch and its static outputs."""

    __slots__ = ("graph", "batch", "loss", "state", "seed_grad", "ring", "drop_seeds")

    def __init__(self, graph, batch, loss, state, seed_grad=None, ring=False, drop_seeds=None):
        self.graph, self.batch, self.loss, self.state = graph, batch, loss, state
        self.seed_grad = seed_grad  # read by the captured backward: kept alive with the graph
        self.ring = ring  # the captured update copies the loss into the engine's loss ring
        # (pool, slots): the dropout seed slots the graph reads, restaged before every replay
        self.drop_seeds = drop_seeds


class ClosureGraph:
    """Host stand-in for a hipGraph (``StepEngine(graph_impl="closure")``, CPU tests): "capture"
    records the step body without running it, ``replay`` re-runs it and copies its loss into the
    static output — so the engine's capture/replay sequence (warm-ups, what runs inside vs after
    the graph, the reducer protocol) executes unchanged on CPU ranks over gloo."""

    def __init__(self):
        self.body = None
        self.loss = None

    def replay(self):
        out = self.body()
        self.loss.copy_(out.detach())


def _to(obj, device):
    if isinstance(obj, torch.Tensor):
        return obj.to(device, non_blocking=True)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(o, device) for o in obj)
    if isinstance(obj, dict):
        return {k: _to(v, device) for k, v in obj.items()}
    return obj


class StepEngine:
    """Executes optimizer steps for ``loss_fn(batch) -> scalar loss``.

    ``optimizer`` is a :class:`perceiver_io_amd.ops.optim.FusedAdamW` (flat buffers; the
    capturable path) or any ``torch.optim.Optimizer`` (eager only).

    With ``graph`` on, a step of ``accumulate`` micro-batches replays ``accumulate - 1``
    "micro" graphs (forward + backward adding into the flat gradient buffer) and one "last"
    graph (forward + backward + the gradient all-reduce + fused AdamW, which also clears the
    gradient it consumes).  Every graph of a step is captured before the step's first
    micro-batch runs (the capture warm-ups clear the gradient buffer).  ``graph_impl``:
    ``"cuda"`` (hipGraph; default on a GPU) or ``"closure"`` (:class:`ClosureGraph`, tests).
    """

    def __init__(self, loss_fn: Callable, optimizer, scheduler=None, reducer=None, device=None,
                 graph: bool = False, accumulate: int = 1, warmup_eager: int = 2, max_graphs: int = 12,
                 state_hooks=None, graph_impl: Optional[str] = None, bucket_update: Optional[bool] = None):
        from ..ops.optim import FusedAdamW

        self.loss_fn = loss_fn
        self.opt = optimizer
        self.sched = scheduler
        self.reducer = reducer
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.fused = isinstance(optimizer, FusedAdamW)
        self.graph_impl = graph_impl or ("cuda" if self.device.type == "cuda" else None)
        self.graph_enabled = bool(graph) and self.fused and self.graph_impl is not None
        self.accumulate = max(1, int(accumulate))
        self.warmup_eager = warmup_eager
        self.max_graphs = max(2, int(max_graphs))
        # state_hooks = (save, restore): side state produced while capturing (e.g. the
        # trainer's logged metric tensors, which are static outputs of that graph) is saved per
        # graph and restored before each replay of it
        self.state_hooks = state_hooks
        self._graphs: "OrderedDict[tuple, _Captured]" = OrderedDict()
        self.captures = 0  # graphs captured so far (evictions included)
        self._loss_ring = None  # (LOSS_RING,) fp32: the returned per-step losses of replayed steps
        self._ring_pos = 0
        self.replays = 0
        self._seed_rng = None  # host stream of the captured graphs' dropout seeds (_stage)
        self._eager_steps = 0
        # every step (eager warmups, capture, replays) runs on ONE dedicated stream: autograd's
        # AccumulateGrad nodes bind to the stream they were created on, and a capture whose
        # accumulations land on another stream silently leaves them outside the graph
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        if self.fused and reducer is not None and reducer.enabled:
            optimizer.grad_scale = reducer.grad_scale()
        self.grad_scale_base = getattr(optimizer, "grad_scale", 1.0)
        # per-bucket optimizer updates: each gradient bucket's AdamW runs right behind its
        # all-reduce on the reducer's side stream (overlapping the rest of the backward), so
        # only the buckets finish() reduces stay on the critical path.  Needs no clipping (a
        # global norm) and no replicated accumulators.
        if bucket_update is None:  # with the reducer's ready points (overlap on) only
            bucket_update = reducer is not None and getattr(reducer, "overlap", False)
        self.bucket_update = bool(bucket_update and self.fused and reducer is not None and reducer.enabled
                                  and optimizer.bucket_updates_ok())
        if self.bucket_update:
            optimizer.bucket_mode = True
            reducer.attach_updater(optimizer.range_update)

    # -- eager -----------------------------------------------------------------------------
    def _arm(self, last: bool):
        r = self.reducer
        if r is not None and r.enabled:
            r.arm() if last else r.disarm()

    def _eager_micro(self, batch, last: bool):
        if last and self.bucket_update:
            self.opt.stage_hyper()  # the bucket updates fire during this backward
        self._arm(last)
        loss = self.loss_fn(batch)
        (loss / self.accumulate if self.accumulate > 1 else loss).backward()
        if last:
            if self.reducer is not None:
                self.reducer.finish()
        return loss

    def _optimizer_step(self):
        if self.fused:
            self.opt.step(staged=self.bucket_update)
        else:
            if self.reducer is not None and self.reducer.enabled:
                for p in self.opt.param_groups[0]["params"]:
                    if p.grad is not None:
                        p.grad.mul_(self.reducer.grad_scale())
            self.opt.step()
        if self.sched is not None:
            self.sched.step()
        if self.reducer is not None:
            self.reducer.flat.zero_grad()  # keep .grad as views of the flat buffer (never None)
        else:
            self.opt.zero_grad()

    # -- graph -----------------------------------------------------------------------------
    @property
    def _self_zeroing(self) -> bool:
        # with the optimizer in the graph, the AdamW kernel clears the gradient it consumes, so a
        # step needs no leading zero fill (gradients are zero between steps on every path: the
        # capture's fill, eager steps' zero_grad, and the previous replay's update)
        return self._opt_in_graph and self.opt.flat.grad_rep is None

    def _capture(self, batch, kind: str) -> _Captured:
        """Capture one step graph for ``batch``'s shape.  ``kind``: ``"last"`` (the optimizer
        step's final micro-batch: backward + all-reduce + AdamW) or ``"micro"`` (an earlier
        micro-batch of an accumulated step: backward only, adding into the gradient)."""
        opt, red = self.opt, self.reducer
        ddp = red is not None and red.enabled
        static = _clone_to(batch, self.device)
        # warm-ups on the capture stream (allocator + lazy init), reducer disarmed: no collective
        # is launched and nothing is left half-done for the captured backward; no optimizer
        # update → nothing to undo but the gradient
        if ddp:
            red.disarm()
        for _ in range(2):
            opt.flat.zero_grad_buffers()
            loss = self.loss_fn(static)
            loss.backward()
            del loss
        opt.flat.zero_grad_buffers()
        last = kind == "last"
        # the backward seed lives outside the graph (autograd would fill a fresh ones tensor
        # inside it on every replay); 1/accumulate averages the micro-batches
        one = torch.full((), 1.0 / self.accumulate, device=self.device)
        in_graph = last and self._opt_in_graph
        zero_inside = last and self.accumulate == 1 and not self._self_zeroing
        # the step's loss leaves through the update kernel (a slot of a device ring, chosen per
        # replay by the staged hyper-parameters) instead of a copy launch after every replay
        ring = in_graph and not opt.bucket_mode
        if ring and self._loss_ring is None:
            self._loss_ring = torch.zeros(LOSS_RING, device=self.device)

        def body():
            if zero_inside:
                opt.flat.zero_grad_buffers()
            if ddp:  # ready points fire inside the graph only when the collectives are captured
                self._arm(in_graph)
            loss = self.loss_fn(static)
            if loss.dim() != 0:  # the 1/accumulate seed averages micro-batches: a scalar loss only
                raise ValueError(f"StepEngine: the loss must be a scalar, got shape {tuple(loss.shape)}")
            loss.backward(one if loss.dtype == one.dtype else one.to(loss.dtype))
            if in_graph:
                if ddp:
                    red.finish()
                if ring:
                    lv = loss.detach()
                    opt.loss_out = (lv if lv.dtype == torch.float32 else lv.float(), self._loss_ring)
                # every replay of this graph is preceded by a staging of the hyper-parameters
                # (_stage), which also zeroes the gradient-norm accumulator
                opt.device_update(zero_grad=self._self_zeroing, norm_staged=True)
                opt.loss_out = None
            return loss

        drop_seeds = None
        if self.graph_impl == "closure":
            g = ClosureGraph()
            g.body = body
            g.loss = loss = torch.zeros((), device=self.device)
        else:
            from ..ops import fused

            g = torch.cuda.CUDAGraph()
            # dropout seeds: static slots staged per replay instead of generator draws in the graph
            fused.begin_static_seeds(self.device)
            try:
                with torch.cuda.graph(g, stream=self.stream):
                    loss = body()
            finally:
                pool, used = fused.end_static_seeds()
            drop_seeds = (pool, used) if used else None
            if ddp:
                red.disarm()
        state = self.state_hooks[0]() if self.state_hooks is not None else None
        self.captures += 1
        return _Captured(g, static, loss, state, one, ring=ring, drop_seeds=drop_seeds)

    def _graph_for(self, batch, kind: str = "last") -> _Captured:
        """The captured step for this batch's shape (captured on first sight, LRU-cached)."""
        key = (kind,) + shape_key(batch)
        ent = self._graphs.get(key)
        if ent is not None:
            self._graphs.move_to_end(key)
            return ent
        while len(self._graphs) >= self.max_graphs:
            _, old = self._graphs.popitem(last=False)
            del old  # its private pool is released with the graph
        ent = self._capture(batch, kind)
        self._graphs[key] = ent
        return ent

    @property
    def num_graphs(self) -> int:
        return len(self._graphs)

    @property
    def _opt_in_graph(self) -> bool:
        r = self.reducer
        return r is None or not r.enabled or getattr(r, "in_graph", False)

    def _kinds(self, n: int):
        return ["micro"] * (n - 1) + ["last"]

    def step(self, batch, ring_view: bool = False):
        """One optimizer step (``accumulate`` micro-batches must be passed as a list); returns the
        step's loss.  A replayed step's loss lives in a slot of a device ring that the captured
        update kernel writes (no copy launch per replay): with ``ring_view=True`` the caller gets
        that slot itself — valid for the next ``LOSS_RING - 1`` steps, for callers that convert it
        right away (Trainer, bench); by default an independent copy, like an eager step's."""
        out = self._step_dispatch(batch)
        if not ring_view and self._loss_ring is not None and out._base is self._loss_ring:
            out = out.clone()
        return out

    def _step_dispatch(self, batch):
        if self.stream is None:
            return self._step(batch)
        batches = batch if (self.accumulate > 1 and isinstance(batch, list)) else [batch]
        if (self.graph_enabled and self._eager_steps >= self.warmup_eager and self._opt_in_graph
                and all((k,) + shape_key(b) in self._graphs for k, b in zip(self._kinds(len(batches)), batches))):
            # a replay needs no autograd stream binding: staging, graph and loss copy go straight
            # onto the caller's stream (a cross-stream event hop costs ~10 µs of GPU idle each way)
            return self._step(batch)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            out = self._step(batch)
        cur.wait_stream(self.stream)
        return out

    def _step(self, batch):
        try:
            return self._step_inner(batch)
        except BaseException:
            if self.reducer is not None:
                self.reducer.reset()
            raise

    def _stage(self, ent, b, hyper: bool):
        if self.graph_impl == "closure":
            _copy_into(ent.batch, b)
            if hyper:
                self.opt.stage_hyper()
        else:
            seeds = None
            if ent.drop_seeds is not None:
                pool, used = ent.drop_seeds
                if self._seed_rng is None:  # host draws: one process-wide stream from torch's seed
                    self._seed_rng = random.Random(torch.initial_seed() ^ 0x5EED5EED)
                seeds = (pool, [self._seed_rng.getrandbits(63) for _ in range(used)])
            _stage_step(ent.batch, b, self.opt if hyper else None, seeds)

    def _step_inner(self, batch):
        batches = batch if (self.accumulate > 1 and isinstance(batch, list)) else [batch]
        if self.graph_enabled and self._eager_steps >= self.warmup_eager:
            kinds = self._kinds(len(batches))
            # every graph of this step first: a capture's warm-ups clear the gradient buffer
            ents = [self._graph_for(b, k) for b, k in zip(batches, kinds)]
            if len(batches) > 1 and not self._self_zeroing:
                self.opt.flat.zero_grad_buffers()
            for i, (b, ent) in enumerate(zip(batches, ents)):
                last = i == len(batches) - 1
                if self.state_hooks is not None:
                    self.state_hooks[1](ent.state)
                # batch copies (+ the optimizer's hyper-parameters before the update graph): one launch
                if last and ent.ring:
                    self.opt.loss_slot = self._ring_pos
                self._stage(ent, b, last and self._opt_in_graph)
                ent.graph.replay()
                self.replays += 1
            if self._opt_in_graph:
                self.opt._step += 1
            else:  # forward+backward replayed; the all-reduce + update eagerly (3 launches)
                if self.bucket_update:
                    self.opt.stage_hyper()
                self.reducer.finish()
                self.opt.step(staged=self.bucket_update)
            if self.sched is not None:
                self.sched.step()
            if ents[-1].ring:  # valid for the next LOSS_RING - 1 steps
                out = self._loss_ring[self._ring_pos]
                self._ring_pos = (self._ring_pos + 1) % LOSS_RING
                return out
            return ents[-1].loss.detach().clone()
        if self.graph_enabled:
            self._eager_steps += 1
        loss = None
        for i, b in enumerate(batches):
            loss = self._eager_micro(_to(b, self.device), i == len(batches) - 1)
        self._optimizer_step()
        return loss.detach()

    def invalidate(self):
        """Drop every captured graph (e.g. after parameters were re-bound)."""
        self._graphs.clear()
