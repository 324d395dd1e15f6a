"""Flat parameter space + fused AdamW (SURVEY K-15, §5.8).

``FlatParameterSpace`` re-homes every trainable parameter into ONE contiguous fp32 buffer
(and its gradient into one fp32 buffer, with a bf16 shadow of the weights for the GEMM
kernels).  Consequences on MI355X:
  * the data-parallel all-reduce is one (or a few bucketed) RCCL call(s) over a flat
    buffer instead of ~190 per-tensor collectives (``parallel/reducer.py``);
  * the optimizer is a single kernel launch over the flat buffers that also refreshes the
    bf16 shadow (no per-step weight casts);
  * zeroing gradients is one memset;
  * parameters flagged ``_pio_replicate`` (the fused attention/MLP layers) are placed first
    and get an 8-way replicated gradient accumulator ``grad_rep`` (8, n_rep): the fused
    backward kernels add their per-row-tile weight-gradient partials into replica
    (tile mod 8), so no address takes more than 1/8 of the tiles' float atomics (same-address
    atomics serialise at the memory side); ``fold()`` adds the replicas into ``grad`` (and
    clears them) once per step, before the all-reduce / optimizer.

``FusedAdamW`` is a ``torch.optim.Optimizer`` (so ``torch.optim.lr_scheduler`` schedulers
such as ``OneCycleLR`` drive it through ``param_groups``) with torch.optim.AdamW semantics
and a torch-compatible ``state_dict`` layout (``exp_avg``/``exp_avg_sq``/``step`` per
parameter), so Lightning-layout checkpoints round-trip.  lr/betas/step live in a small
device tensor refreshed before each step, which keeps the update capturable in a hipGraph.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional

import torch

from . import emulation, ext

ALIGN = 64  # elements; keeps every parameter view 256-byte aligned


GRAD_REPLICAS = 8  # matches kGradReplicas in csrc/rowgemm.hip


class FlatParameterSpace:
    def __init__(self, params: Iterable[torch.nn.Parameter], with_shadow: Optional[bool] = None,
                 replicate: Optional[bool] = None):
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dev = params[0].device
        self.device = dev
        if replicate is None:
            # the replicas only serve the in-kernel float-atomic gradient path; with per-tile
            # weight-gradient slabs (ops.fused.WGRAD_SLAB) they would stay zero
            from .fused import WGRAD_SLAB

            replicate = dev.type == "cuda" and not WGRAD_SLAB
        rep = [p for p in params if replicate and getattr(p, "_pio_replicate", False)]
        rep_ids = {id(p) for p in rep}
        # replicated parameters first (one contiguous region), then the rest in module order
        self.params: List[torch.nn.Parameter] = rep + [p for p in params if id(p) not in rep_ids]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.n_rep = self.offsets[len(rep)] if len(rep) < len(self.params) else off
        if not rep:
            self.n_rep = 0
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad_rep = torch.zeros(GRAD_REPLICAS, self.n_rep, dtype=torch.float32, device=dev) if rep else None
        if with_shadow is None:
            with_shadow = dev.type == "cuda"
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=dev) if with_shadow else None
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                self.data[o:o + n].copy_(p.detach().reshape(-1).float())
                p.data = self.data[o:o + n].view_as(p)
                p.grad = self.grad[o:o + n].view_as(p)
                p._pio_flat = True  # its gradient is a view of this flat buffer (ops/fused.py in-place paths)
                if self.grad_rep is not None and o < self.n_rep:
                    p._pio_grad_rep = self.grad_rep[:, o:o + n]  # (8, numel) replica view
        if self.shadow is not None:
            from .fused import weight_cache

            for p, o in zip(self.params, self.offsets):
                weight_cache.bind(p, self.shadow[o:o + p.numel()].view(p.shape))

    def fold(self):
        """grad[:n_rep] += Σ replicas; replicas ← 0 (no-op without replicated parameters)."""
        if self.grad_rep is None:
            return
        K = ext.require() if self.device.type == "cuda" else emulation
        K.fold_replicas(self.grad, self.grad_rep)

    def views(self, buf: torch.Tensor):
        return [buf[o:o + p.numel()].view(p.shape) for p, o in zip(self.params, self.offsets)]

    def zero_grad_buffers(self):
        """Zero the gradient buffer and its replicas (capturable; no Python-side view fixes)."""
        self.grad.zero_()
        if self.grad_rep is not None:
            self.grad_rep.zero_()

    def zero_grad(self):
        self.zero_grad_buffers()
        # re-attach views autograd may have replaced (e.g. a grad that was set to None)
        for p, o in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != self.grad[o:o + 1].data_ptr():
                p.grad = self.grad[o:o + p.numel()].view_as(p)

    def check_views(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad[o:o + 1].data_ptr()
                   for p, o in zip(self.params, self.offsets))

    def bucket_ranges(self, bucket_bytes: int, hi: Optional[int] = None):
        """Split [0, hi) (default: the whole buffer) into contiguous ranges of about
        ``bucket_bytes`` at parameter boundaries, in reverse parameter order (gradients of late
        parameters are produced first in backward)."""
        cap = max(ALIGN, bucket_bytes // 4)
        hi = self.numel if hi is None else hi
        ranges = []
        for o in reversed(self.offsets):
            if o >= hi:
                continue
            if hi - o >= cap:
                ranges.append((o, hi))
                hi = o
        if hi > 0:
            ranges.append((0, hi))
        return ranges


class _HostRing:
    """Pinned host staging slots for per-step device hyper-parameters (no reuse before the
    copy that read a slot has completed)."""

    def __init__(self, n: int, width: int, device):
        self.slots = [torch.zeros(width, dtype=torch.float32).pin_memory() for _ in range(n)]
        self.events = [None] * n
        self.i = 0

    def push(self, values, dst: torch.Tensor):
        i = self.i
        self.i = (self.i + 1) % len(self.slots)
        if self.events[i] is not None:
            self.events[i].synchronize()
        s = self.slots[i]
        for j, v in enumerate(values):
            s[j] = float(v)
        dst.copy_(s, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev


class FusedAdamW(torch.optim.Optimizer):
    """AdamW over a :class:`FlatParameterSpace` in one kernel (HIP) or its emulation (CPU)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 amsgrad: bool = False, max_grad_norm: float = 0.0, flat: Optional[FlatParameterSpace] = None):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by the fused optimizer")
        params = list(params)
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdamW supports a single parameter group")
        # always with the bf16 shadow the fused executor reads its GEMM operands from (also for the
        # CPU emulation: re-homed parameters do not share the flat buffer's version counter, so a
        # version-keyed weight cache would never see the in-place update)
        self.flat = flat if flat is not None else FlatParameterSpace(self.param_groups[0]["params"], with_shadow=True)
        dev = self.flat.device
        self.exp_avg = torch.zeros(self.flat.numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.flat.numel, dtype=torch.float32, device=dev)
        self.hyper = torch.zeros(8, dtype=torch.float32, device=dev)
        self.max_grad_norm = float(max_grad_norm)
        # the gradient's sum of squares as fixed-order per-block partials (sumsq → adamw norm_part):
        # no atomics, so the clip factor is bitwise reproducible in every mode
        self.norm_part = torch.zeros(512, dtype=torch.float32, device=dev) if self.max_grad_norm > 0 else None
        self.l2 = False  # decoupled decay (AdamW); FusedAdam sets the coupled L2 form
        self._step = 0
        self._ring = _HostRing(8, 8, dev) if dev.type == "cuda" else None
        self.grad_scale = 1.0
        # bucket mode (set by the step engine with a data-parallel reducer): each gradient bucket
        # is updated by range_update right after its all-reduce lands, on the reducer's side
        # stream, so device_update has nothing left to do
        self.bucket_mode = False
        # set by the step engine around a captured update: the kernel also copies the step's
        # loss (loss_out[0]) into loss_out[1][hyper[7]] (see StepEngine's loss ring)
        self.loss_out = None
        self.loss_slot = 0

    # -- the update ---------------------------------------------------------------------
    def hyper_values(self):
        """lr / step / betas of the NEXT update (and the step engine's loss-ring slot), in
        ``self.hyper``'s layout."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        return [float(g["lr"]), float(self._step + 1), 0.0, float(b1), float(b2), 0.0, 0.0, float(self.loss_slot)]

    def stage_hyper(self):
        """Write lr / step / betas for the NEXT update into device memory (outside any graph)."""
        vals = self.hyper_values()
        if self._ring is not None:
            self._ring.push(vals, self.hyper)
        else:
            self.hyper.copy_(torch.tensor(vals))

    def bucket_updates_ok(self) -> bool:
        """Per-bucket updates are exact only without a global gradient norm (clipping) and without
        replicated gradient accumulators (a later fold would add into an updated range)."""
        return self.max_grad_norm <= 0 and self.flat.grad_rep is None

    def range_update(self, lo: int, hi: int):
        """Fused AdamW over flat elements [lo, hi) only (the same per-element arithmetic as the
        whole-buffer kernel, so a step made of range updates is bitwise the full update); the
        gradient range is cleared as it is consumed.  Reads the hyper-parameters already staged
        for this step."""
        K = ext.require() if self.flat.device.type == "cuda" else emulation
        g = self.param_groups[0]
        f = self.flat
        K.adamw(f.data[lo:hi], f.grad[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi],
                None if f.shadow is None else f.shadow[lo:hi], self.hyper, g["eps"], g["weight_decay"], 0.0,
                self.grad_scale, l2=self.l2, zero_grad=True)

    def device_update(self, zero_grad: bool = False, norm_staged: bool = False):
        """The capturable part: (grad-norm) + fused AdamW kernel over the flat buffers.
        ``zero_grad``: the kernel clears the gradient as it consumes it (flat buffers without
        replicas only; the step engine's captured step then skips its leading zero fill).
        In bucket mode the reducer has already updated every bucket: nothing to do."""
        if self.bucket_mode:
            return
        K = ext.require() if self.flat.device.type == "cuda" else emulation
        g = self.param_groups[0]
        self.flat.fold()
        if self.max_grad_norm > 0:
            K.sumsq(self.flat.grad, self.norm_part)
        lo = self.loss_out
        K.adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.flat.shadow, self.hyper,
                g["eps"], g["weight_decay"], self.max_grad_norm, self.grad_scale, l2=self.l2,
                zero_grad=zero_grad and self.flat.grad_rep is None,
                loss_src=None if lo is None else lo[0], loss_ring=None if lo is None else lo[1],
                norm_part=self.norm_part)

    @torch.no_grad()
    def step(self, closure=None, staged: bool = False):
        loss = closure() if closure is not None else None
        if not staged:
            self.stage_hyper()
        self.device_update()
        self._step += 1
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    # -- torch-compatible state dict ------------------------------------------------------
    def state_dict(self):
        sd = super().state_dict()
        state = {}
        ea, es = self.flat.views(self.exp_avg), self.flat.views(self.exp_avg_sq)
        for i in range(len(self.flat.params)):
            state[i] = {"step": torch.tensor(float(self._step)), "exp_avg": ea[i].clone(), "exp_avg_sq": es[i].clone()}
        sd["state"] = state
        return sd

    def load_state_dict(self, state_dict):
        state = state_dict.get("state", {})
        groups = state_dict["param_groups"]
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
        ea, es = self.flat.views(self.exp_avg), self.flat.views(self.exp_avg_sq)
        step = 0
        for i, st in state.items():
            i = int(i)
            if "exp_avg" in st:
                ea[i].copy_(st["exp_avg"])
                es[i].copy_(st["exp_avg_sq"])
            step = int(float(st.get("step", 0)))
        self._step = step


class FusedAdam(FusedAdamW):
    """``torch.optim.Adam`` semantics (coupled L2: ``weight_decay · p`` joins the gradient after
    clipping) in the same single fused kernel — the optimizer of the LArTPC experiment
    (reference ``run.py:134``: ``Adam(lr=1e-3, weight_decay=1e-4)`` + ``clip_grad_norm_(10)``).
    Parameters whose gradient is identically zero still decay, exactly as torch.optim.Adam does
    for parameters that took part in the backward; leave parameters that never receive a
    gradient (torch skips ``grad is None``) out of ``params``."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, max_grad_norm: float = 0.0, flat: Optional[FlatParameterSpace] = None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         max_grad_norm=max_grad_norm, flat=flat)
        self.l2 = True
