"""Data-parallel gradient reducer over the flat gradient buffer (SURVEY C-01..C-03, §5.8).

Replaces the DDP Reducer the reference gets from Lightning (``trainer.yaml:47``: every gradient
averaged over the ranks on every step):
  * parameters and buffers are broadcast once from rank 0 as flat tensors (C-01); the
    deterministic Fourier position-encoding buffer is *not* re-broadcast every step (C-02);
  * gradients live in ONE contiguous fp32 buffer (``ops.optim.FlatParameterSpace``), reduced by
    a few large RCCL all-reduces instead of per-parameter buckets.  Per-step gradient volume is
    4–11 MB, so on xGMI (point-to-point links, ring all-reduce bound by one link per hop) the
    collective is latency-bound: 3–4 buckets, not DDP's 25 MB-bucket machinery;
  * the average (÷ world) is folded into the fused optimizer's gradient scale (no extra pass);
  * overlap with the backward through READY POINTS: identity autograd nodes placed on a tensor
    whose gradient arrives only after a known flat range of parameter gradients is final
    (``bucket_ready_point``).  Their backward launches that range's all-reduce on a side HIP
    stream while the rest of the backward runs:
      - ``"decoder"`` on the decoder's input: the decoder + output head (the flat buffer's tail);
      - ``"layer_n"`` on the input of the weight-shared ``layer_n``'s first application: all of
        ``layer_n`` except its cross-attention query path (the fused executor runs that
        LN + Q-projection backward inside ``layer_1``'s self-attention block backward,
        ``ops/fused.py`` ``_LOOKAHEAD["bwd_q"]``), i.e. from the K/V part of its in-projection
        bias to its last parameter.
    ``finish()`` reduces the remaining buckets (embedding, ``layer_1``, latents, the layer_n
    query path) and joins the side stream.

Step protocol (enforced, so a stale launch can never leak into a later step or a graph):
    arm()      before the forward of the LAST micro-batch of an optimizer step — ready points
               fire only while armed (with gradient accumulation the earlier micro-batches'
               backwards launch nothing: their gradients are not final yet);
    backward   ready points launch their buckets (each at most once; a second hit is an error);
    finish()   launches every bucket not launched yet, joins, disarms.
While a hipGraph capture is in progress, ``arm()`` only arms when the collectives are captured
into the graph (``in_graph``: RCCL capturable on this node, probed once by
``dist.graph_collectives_ok``); otherwise the captured backward launches nothing and
``finish()`` runs eagerly after each replay.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

_ACTIVE: List["FlatGradReducer"] = []


class _ReadyFn(torch.autograd.Function):
    """Identity whose backward launches the bucket of one ready point.

    Applied to a tensor *before* any op of the covered parameters is recorded.  The autograd
    engine runs this node only once the gradient of its output is complete, i.e. after every
    node that consumed the output; the covered parameters' AccumulateGrad nodes run as soon as
    their inputs are ready (highest priority), and the fused kernels' deferred weight-gradient
    slab reductions are flushed first (``ops.fused.flush_pending``)."""

    @staticmethod
    def forward(ctx, x, red, name):
        ctx.red, ctx.name = red, name
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.red.point_reached(ctx.name)
        return g, None, None


def ready_point_armed(module: torch.nn.Module, name: str) -> bool:
    """Whether ready point ``name`` of ``module`` would fire in this step's backward (an armed
    reducer planned it): gradients of that range must then be final when the point's gradient
    arrives, so a caller may not defer part of their computation past it."""
    return any(red.armed and red.owns_point(module, name) for red in _ACTIVE)


def bucket_ready_point(x: torch.Tensor, module: torch.nn.Module, name: str) -> torch.Tensor:
    """Mark ``x`` as ready point ``name`` of the armed reducer that planned ``module``."""
    if not _ACTIVE or not torch.is_grad_enabled() or not x.requires_grad:
        return x
    for red in reversed(_ACTIVE):
        if red.owns_point(module, name):
            if not red.armed:
                return x
            return _ReadyFn.apply(x, red, name)
    return x


def _capturing(device) -> bool:
    return device.type == "cuda" and torch.cuda.is_current_stream_capturing()


class FlatGradReducer:
    def __init__(self, flat, bucket_bytes: Optional[int] = None, overlap: Optional[bool] = None,
                 in_graph: Optional[bool] = None, wire_dtype: Optional[torch.dtype] = None, force: bool = False):
        self.flat = flat
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        # force: run the collectives even for a 1-rank group (tests of the capture mechanics on one GPU)
        self.force = bool(force) and dist.is_available() and dist.is_initialized()
        # bucket_bytes=None: 4 MB buckets with overlap, the whole buffer in one all-reduce without
        # (an explicit size keeps the overlapped layout, ready-point ranges included, also when
        # overlap is off: the two paths then add in the same order — bit-comparable)
        self._one_bucket = bucket_bytes is None
        bucket_bytes = 4 << 20 if bucket_bytes is None else bucket_bytes
        self.bucket_bytes = bucket_bytes
        self.buckets: List[Tuple[int, int]] = flat.bucket_ranges(bucket_bytes)
        self.points: Dict[str, int] = {}          # ready point → bucket index
        self._point_modules: Dict[str, int] = {}  # ready point → id() of the module it was planned on
        # overlap needs every parameter gradient to land in flat.grad directly (no 8-way replicas
        # that a later fold() would still add into an early bucket's range)
        # overlap=None → off: the inline path — ONE all-reduce over the whole flat gradient on the
        # compute stream after the backward (inside the step graph where RCCL is capturable), then
        # one fused AdamW.  Measured on one MI355X with the collectives forced on (1-rank RCCL,
        # profiles/r6_reducer_ab.md): the side-stream ready points + per-bucket AdamW expose
        # ≈150 µs per headline step (cross-queue gaps, contention, five AdamW launches), the
        # inline path ≈5 µs; at 4–11 MB of gradients per step an 8-GPU xGMI ring all-reduce
        # costs less than that overlap machinery, so it is not worth hiding.  overlap=True keeps
        # the ready points (tests, A/B: bench.py --overlap on).
        if overlap is None:
            overlap = False
        self.overlap = bool(overlap) and getattr(flat, "grad_rep", None) is None
        self._one_bucket = self._one_bucket and not self.overlap
        if self._one_bucket:  # one large message: the ring pays its per-hop latency once
            self.bucket_bytes = 256 << 20
            self.buckets = flat.bucket_ranges(self.bucket_bytes)
        self.wire_dtype = wire_dtype
        self.on_gpu = flat.device.type == "cuda"
        self._side = torch.cuda.Stream(device=flat.device) if (self.on_gpu and self.overlap) else None
        self._counts = [0] * len(self.buckets)
        self._armed = False
        # updater(lo, hi): the optimizer's range update, run right after a bucket's all-reduce on
        # the same (side) stream — the whole update overlaps the backward except for the buckets
        # finish() reduces (attach_updater)
        self.updater = None
        self.early_launches = 0  # buckets launched from a backward (tests / diagnostics)
        self.launch_log: List[str] = []  # names of the ready points that fired, in order (tests)
        if in_graph is None:
            from .dist import graph_collectives_ok

            # the side-stream ready points are never captured (auto mode): a step graph holding
            # RCCL work forked onto a second stream aborted at capture end, without a message,
            # in one of several runs of the same test (rounds 5 and 6); the overlapped path keeps
            # its collectives outside the graph, the default (inline) path is single-stream
            in_graph = self.enabled and self.on_gpu and not self.overlap and graph_collectives_ok(flat.device)
        self.in_graph = bool(in_graph)
        if self.enabled:
            _ACTIVE.append(self)

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.force

    @property
    def armed(self) -> bool:
        return self._armed

    def close(self):
        """Unregister (end of a fit / bench): a stale reducer must never be the target of a later
        model's ready points."""
        if self in _ACTIVE:
            _ACTIVE.remove(self)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- buckets -------------------------------------------------------------------------
    def _param_range(self, params, lo_param=None, lo_extra: int = 0) -> Optional[Tuple[int, int]]:
        """Flat range [lo, hi) covering exactly ``params`` (contiguous in the buffer), optionally
        starting ``lo_extra`` elements into ``lo_param``; None if they are not contiguous."""
        ids = {id(p) for p in params}
        idx = [i for i, p in enumerate(self.flat.params) if id(p) in ids]
        if not idx or idx != list(range(idx[0], idx[-1] + 1)):
            return None
        offs = self.flat.offsets
        last = idx[-1]
        hi = offs[last + 1] if last + 1 < len(offs) else self.flat.numel
        lo = offs[idx[0]]
        if lo_param is not None:
            j = next((i for i in idx if self.flat.params[i] is lo_param), None)
            if j is None:
                return None
            lo = offs[j] + (lo_extra + 3) // 4 * 4  # 4-element aligned: the vector update kernel's ranges
        return (lo, hi) if hi > lo else None

    def set_ready_ranges(self, ranges: Dict[str, Tuple[Tuple[int, int], torch.nn.Module]]):
        """Ready points ``name → ((lo, hi), module)``: disjoint flat ranges reduced when the
        backward reaches the point; the complement is split into ``bucket_bytes`` buckets that
        ``finish()`` reduces."""
        items = sorted(((r, n, m) for n, (r, m) in ranges.items()), key=lambda t: -t[0][0])
        for (a, _, _), (b, _, _) in zip(items, items[1:]):
            if b[1] > a[0]:
                raise ValueError("ready-point ranges overlap")
        self.buckets, self.points, self._point_modules = [], {}, {}
        for (lo, hi), name, mod in items:
            self.points[name] = len(self.buckets)
            self._point_modules[name] = id(mod)
            self.buckets.append((lo, hi))
        # the complement, highest offsets first (late parameters' gradients are produced first)
        hi = self.flat.numel
        gaps = []
        for (lo_r, hi_r), _, _ in items:
            if hi_r < hi:
                gaps.append((hi_r, hi))
            hi = lo_r
        if hi > 0:
            gaps.append((0, hi))
        cap = max(64, self.bucket_bytes // 4 // 64 * 64)  # bucket boundaries stay 64-element (256-B) aligned
        for lo, hi in gaps:
            while hi - lo > cap:
                self.buckets.append((hi - cap, hi))
                hi -= cap
            self.buckets.append((lo, hi))
        self._counts = [0] * len(self.buckets)

    def plan(self, model) -> Dict[str, Tuple[int, int]]:
        """Ready points for a Perceiver model (anything with ``.decoder`` and/or ``.encoder``):
        ``"decoder"`` and, for a weight-shared encoder (``layer_n``), ``"layer_n"`` and
        ``"layer_1_sa"`` (layer_1's self-attention block).  Returns the
        planned flat ranges (empty when nothing can overlap, e.g. a frozen encoder's decoder-only
        training keeps one bucket)."""
        ranges = {}
        dec = getattr(model, "decoder", None)
        if isinstance(dec, torch.nn.Module):
            r = self._param_range([p for p in dec.parameters() if p.requires_grad])
            if r is not None:
                ranges["decoder"] = (r, dec)
        enc = getattr(model, "encoder", None)
        lay = getattr(enc, "layer_n", None) if isinstance(enc, torch.nn.Module) else None
        if lay is not None:
            ps = [p for p in lay.parameters() if p.requires_grad]
            try:
                mha = lay[0].attn.attention.attention
                bias, c = mha.in_proj_bias, mha.embed_dim
            except (AttributeError, IndexError, TypeError):
                bias = None
            if ps and bias is not None and bias.requires_grad:
                # everything of layer_n from the K/V part of its in-projection bias on (the query
                # path before it finishes inside layer_1's backward on the fused path)
                r = self._param_range(ps, lo_param=bias, lo_extra=c)
                if r is not None:
                    ranges["layer_n"] = (r, enc)
        l1 = getattr(enc, "layer_1", None) if isinstance(enc, torch.nn.Module) else None
        blk = l1[1] if isinstance(l1, torch.nn.Sequential) and len(l1) > 1 else None
        if blk is not None and lay is not None:
            # layer_1's self-attention block: final once the backward leaves it, but for its first
            # layer's LN1 + QKV projection (on the fused path the preceding cross layer's kernel
            # computes that backward) — the range starts at that layer's out-projection
            bps = [p for p in blk.parameters() if p.requires_grad]
            try:
                first_out = blk[0][0].module.attention.attention.out_proj.weight
            except (AttributeError, IndexError, TypeError):
                first_out = None
            if bps and first_out is not None and first_out.requires_grad:
                r = self._param_range(bps, lo_param=first_out)
                if r is not None:
                    ranges["layer_1_sa"] = (r, enc)
        if not self.overlap:
            # overlap off: no ready points; the whole buffer in one bucket (default), or the
            # overlapped layout when a bucket size was given (bit-comparable A/B)
            if not self._one_bucket:
                self.set_ready_ranges(ranges)
            self.points, self._point_modules = {}, {}
            return {}
        self.set_ready_ranges(ranges)
        return {k: v[0] for k, v in ranges.items()}

    def set_early_params(self, params: Iterable[torch.nn.Parameter], module: Optional[torch.nn.Module] = None):
        """Compatibility: one ``"decoder"`` ready point over ``params`` (a contiguous range)."""
        params = list(params)
        r = self._param_range([p for p in params if p.requires_grad])
        if r is None:
            return
        if module is None:
            raise ValueError("set_early_params needs the module whose forward places the ready point")
        self.set_ready_ranges({"decoder": (r, module)})
        if not self.overlap:
            self.points, self._point_modules = {}, {}

    @property
    def early(self) -> Optional[Tuple[int, int]]:
        i = self.points.get("decoder")
        return self.buckets[i] if i is not None else None

    def owns_point(self, module, name: str) -> bool:
        return self._point_modules.get(name) == id(module)

    def overlap_ready(self) -> bool:
        return self.enabled and self.overlap and bool(self.points)

    def broadcast_parameters(self, module: torch.nn.Module, src: int = 0):
        """C-01: one broadcast of the flat parameter buffer + remaining buffers."""
        if not self.enabled:
            return
        dist.broadcast(self.flat.data, src=src)
        flat_ptrs = {p.data_ptr() for p in self.flat.params}
        for name, b in module.named_buffers():
            if name.endswith("position_encoding"):
                continue  # deterministic (C-02)
            dist.broadcast(b, src=src)
        for p in module.parameters():
            if p.data_ptr() not in flat_ptrs:
                dist.broadcast(p.data, src=src)

    # -- the step protocol ----------------------------------------------------------------
    def _join(self):
        if self._side is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)

    def arm(self):
        """Before the forward of an optimizer step's last micro-batch."""
        if any(self._counts):
            raise RuntimeError("FlatGradReducer.arm: buckets of a previous backward were never finished "
                               f"(launched: {[i for i, c in enumerate(self._counts) if c]})")
        capturing = _capturing(self.flat.device)
        self._armed = self.overlap_ready() and (not capturing or self.in_graph)

    def disarm(self):
        self._armed = False

    def reset(self):
        """Abandon a step (e.g. after an exception inside it): join outstanding launches, clear."""
        if any(self._counts) and not _capturing(self.flat.device):
            self._join()
        self._counts = [0] * len(self.buckets)
        self._armed = False

    def _reduce(self, lo: int, hi: int):
        g = self.flat.grad[lo:hi]
        if self.wire_dtype is not None and self.wire_dtype != g.dtype:
            w = g.to(self.wire_dtype)
            dist.all_reduce(w)
            g.copy_(w)
        else:
            dist.all_reduce(g)

    def attach_updater(self, fn) -> None:
        """Update each bucket's parameters as soon as its all-reduce lands (``fn(lo, hi)``, e.g.
        :meth:`FusedAdamW.range_update`); None detaches."""
        self.updater = fn

    def _launch(self, bucket: int, flush: bool = False):
        if _capturing(self.flat.device) and not self.in_graph:
            raise RuntimeError("FlatGradReducer: a collective inside a hipGraph capture on a node where the "
                               "collectives are not capturable (in_graph=False)")
        self._counts[bucket] += 1
        lo, hi = self.buckets[bucket]
        from ..ops.fused import flush_pending

        if self._side is not None:
            run_side = None
            if flush:  # the covered kernels' deferred slab reductions, ahead of the collective:
                # those entirely inside the bucket on the side stream, the rest (still being
                # accumulated on the main stream) on the main stream before the fork
                base = self.flat.grad.data_ptr()

                def inside(d, lo=lo, hi=hi, base=base):
                    off = (d.data_ptr() - base) // d.element_size()
                    return d.dtype == self.flat.grad.dtype and lo <= off and off + d.numel() <= hi

                run_side = flush_pending(self._side, inside)
            self._side.wait_stream(torch.cuda.current_stream(self.flat.device))
            if run_side is not None:
                run_side()
            with torch.cuda.stream(self._side):
                self._reduce(lo, hi)
                if self.updater is not None:
                    self.updater(lo, hi)
        else:
            if flush:
                flush_pending()
            self._reduce(lo, hi)
            if self.updater is not None:
                self.updater(lo, hi)

    def point_reached(self, name: str):
        """Backward reached ready point ``name``: its bucket is final → launch it."""
        if not (self._armed and self.enabled):
            return
        i = self.points[name]
        if self._counts[i]:
            raise RuntimeError(f"FlatGradReducer: ready point {name!r} reached twice in one backward")
        self.early_launches += 1
        self.launch_log.append(name)
        # the deferred weight-gradient slab reductions of the covered kernels run first, on the
        # side stream (the bucket's only consumer) when there is one
        self._launch(i, flush=True)

    def finish(self):
        """All remaining buckets, then join the side stream; every bucket exactly once."""
        if not self.enabled:
            self._armed = False
            return
        self.flat.fold()  # replicated fused-layer gradients → grad before they are reduced
        for i in range(len(self.buckets)):
            if not self._counts[i]:
                self._launch(i)
        self._join()
        if any(c != 1 for c in self._counts):
            raise RuntimeError(f"FlatGradReducer.finish: bucket launch counts {self._counts} (each must be 1)")
        self._counts = [0] * len(self.buckets)
        self._armed = False

    def grad_scale(self) -> float:
        return 1.0 / self.world


def params_in_sync(flat_or_params, src: int = 0) -> float:
    """max |p − p_rank0| over every parameter (all ranks agree on the value; 0.0 = bitwise in
    sync).  One broadcast of the flat buffer + one max all-reduce — a cheap end-of-run check."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
        return 0.0
    if isinstance(flat_or_params, torch.Tensor):
        mine = flat_or_params.detach().float().reshape(-1)
    elif hasattr(flat_or_params, "data") and isinstance(flat_or_params.data, torch.Tensor):
        mine = flat_or_params.data.detach().float().reshape(-1)
    else:
        mine = torch.cat([p.detach().float().reshape(-1) for p in flat_or_params])
    ref = mine.clone()
    dist.broadcast(ref, src=src)
    d = (mine - ref).abs().max().reshape(1)
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    return float(d.item())
