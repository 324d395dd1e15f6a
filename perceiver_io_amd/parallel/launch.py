"""Single-node launcher: one child process per GPU (the role Lightning's DDP spawner plays
for ``--trainer.devices=-1``).

The parent never initialises the GPU (it only counts devices), starts N children with the
torchrun environment (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``,
``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``) and returns the worst exit code.  If one child
fails the others are terminated (their process group), so a crashed rank cannot leave the
rest hanging in a collective.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_list(v: str) -> int:
    return len([t for t in v.split(",") if t.strip() != ""])


def topology_gpu_count(topo: str = "/sys/class/kfd/kfd/topology/nodes", dri: str = "/dev/dri") -> Optional[int]:
    """GPUs of the KFD topology that this process can open, or None without a topology.

    A node counts when it has SIMDs (``simd_count > 0``) AND its render node
    ``{dri}/renderD<drm_render_minor>`` is readable and writable — the filter ROCr applies: a
    container given only some of the host's render nodes still lists every host GPU in the
    topology, and HIP skips the ones it cannot open."""
    if not os.path.isdir(topo):
        return None
    n = 0
    for node in os.listdir(topo):
        try:
            with open(os.path.join(topo, node, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            if int(props.get("simd_count", "0")) <= 0:
                continue
            minor = int(props["drm_render_minor"])
        except (OSError, ValueError, KeyError):
            continue
        if os.access(os.path.join(dri, f"renderD{minor}"), os.R_OK | os.W_OK):
            n += 1
    return n


def gpu_count() -> int:
    """Number of GPUs this process would see, WITHOUT initialising HIP in this process (the
    launcher parent must hold no GPU state when it starts the ranks).

    Order: an explicit ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
    list; else the openable GPU nodes of the KFD topology (``topology_gpu_count``); else a
    short-lived child process that asks torch (its HIP runtime dies with it)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return _visible_list(v)
    n = topology_gpu_count()
    if n:
        return n
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def spawn(nprocs: int, cmd: List[str], env: Optional[dict] = None, port: Optional[int] = None) -> int:
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(port or base.get("MASTER_PORT") or free_port())
    base["WORLD_SIZE"] = str(nprocs)
    base["LOCAL_WORLD_SIZE"] = str(nprocs)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
    rc = 0
    try:
        alive = set(range(nprocs))
        while alive:
            for i in list(alive):
                c = procs[i].poll()
                if c is None:
                    continue
                alive.discard(i)
                if c != 0:
                    rc = rc or c
                    for j in alive:  # take the others down: a lone rank would hang in RCCL
                        try:
                            os.killpg(procs[j].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        rc = 130
    return rc


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="python -m perceiver_io_amd.parallel.launch --nproc N script.py [args]")
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    sys.exit(spawn(a.nproc, [sys.executable] + a.cmd))


if __name__ == "__main__":
    main()
