"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL.

Reference: Lightning ``ddp_find_unused_parameters_false`` (``scripts/trainer.yaml:47``) —
one process per device, NCCL process group.  Here: torchrun-style environment
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``); backend ``nccl``
(= RCCL over xGMI on ROCm) for GPU ranks, ``gloo`` for CPU ranks (tests).  The default
rendezvous address is 127.0.0.1 (single node).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def info() -> DistInfo:
    return _INFO


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: str | None = None, timeout_s: float = 1800.0, device_type: str | None = None) -> DistInfo:
    """Initialise the default process group from the environment (idempotent)."""
    global _INFO
    ws = env_world_size()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if ws <= 1:
        _INFO = DistInfo(rank=0, local_rank=0, world_size=1, backend="none")
        return _INFO
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if backend is None:  # PERCEIVER_DIST_BACKEND=gloo: rehearse GPU ranks over gloo (e.g. several on one GPU)
        backend = os.environ.get("PERCEIVER_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    # the host driver only supports dmabuf IPC (RCCL / CUDA-tensor sharing across processes)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if device_type == "cuda":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    elif "OMP_NUM_THREADS" not in os.environ:
        # CPU ranks of one node share its cores: without a split every rank's intra-op pool spans
        # all of them, and the oversubscribed, spinning pools run ~10x slower than split ones
        local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, local_ws)))
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(**kw)
    _INFO = DistInfo(rank=rank, local_rank=local, world_size=ws, backend=backend)
    return _INFO


_GRAPH_COLL = {}


def graph_collectives_ok(device) -> bool:
    """Can RCCL collectives be captured in a hipGraph on this node?  Probed once per device:
    every rank captures a tiny all-reduce on a side stream, the ranks agree (eager all-reduce of
    the capture status) before anyone replays, the replay's result is checked, and the ranks
    agree again.  ``PERCEIVER_GRAPH_COLLECTIVES=0/1`` forces the answer.  Never true for gloo."""
    env = os.environ.get("PERCEIVER_GRAPH_COLLECTIVES")
    if _INFO.backend != "nccl" or not (dist.is_available() and dist.is_initialized()):
        return False
    if env is not None:
        return env not in ("0", "", "false")
    device = torch.device(device)
    if device in _GRAPH_COLL:
        return _GRAPH_COLL[device]
    ws = _INFO.world_size
    t = torch.ones(64, device=device)
    side = torch.cuda.Stream(device=device)
    g = None
    captured = 1.0
    try:
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            dist.all_reduce(t)  # warm the communicator outside the capture
        torch.cuda.synchronize(device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            dist.all_reduce(t)
    except Exception:  # noqa: BLE001 - any capture failure means "not capturable"
        captured = 0.0
        # torch.cuda.graph ends the capture when the with-block exits, also on an exception; a
        # capture left open half-way would poison the side stream (and, in global capture mode,
        # every later launch of the process): end it here before anything else runs
        with torch.cuda.stream(side):
            if g is not None and torch.cuda.is_current_stream_capturing():
                try:
                    g.capture_end()
                except Exception:  # noqa: BLE001 - an invalidated capture still ends capture mode
                    pass
        g = None
    flag = torch.tensor([captured], device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    ok = bool(flag.item() > 0.5)
    if ok:
        t.fill_(1.0)
        torch.cuda.synchronize(device)
        g.replay()
        torch.cuda.synchronize(device)
        good = float(torch.allclose(t, torch.full_like(t, float(ws))))
        flag = torch.tensor([good], device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item() > 0.5)
    _GRAPH_COLL[device] = ok
    return ok


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t.item()) / _INFO.world_size


def broadcast_object(obj, src: int = 0):
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
