"""Build the in-tree HIP extension ``perceiver_io_amd/_C*.so`` for gfx950.

Kernels (``*.hip``) are compiled with ``hipcc --offload-arch=gfx950`` and contain no
PyTorch headers (fast, parallel, cached by content hash); only ``binding.cpp`` sees
the torch headers (host compiler).  No hipify pass, no JIT cache outside the tree:
the resulting ``.so`` travels with the repository snapshot to the GPU box.

    python -m perceiver_io_amd.csrc.build [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
BUILD = PKG.parent / "build" / "csrc"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


# MFMA results in VGPRs (no AGPR staging) for the translation units whose kernels post-process
# accumulators with VALU (softmax, LayerNorm, GELU) and fit 256 VGPRs; rowgemm.hip keeps the
# default (its 160-channel LN-linear backward would spill without the AGPR file)
_VGPR_FORM = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
PER_FILE_FLAGS = {"chain.hip": _VGPR_FORM, "attention_pe.hip": _VGPR_FORM, "ce_head.hip": _VGPR_FORM,
                  "persist.hip": _VGPR_FORM}


def _torch_paths():
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths()
    libdir = os.path.join(os.path.dirname(ce.__file__), "..", "lib")
    return inc, os.path.abspath(libdir)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"command failed ({r.returncode}): {cmd[0]} … {cmd[-1]}")
    return r.stdout


def _digest(paths, flags):
    h = hashlib.sha256(" ".join(flags).encode())
    for p in paths:
        h.update(Path(p).read_bytes())
    return h.hexdigest()[:16]


def ext_path(name: str = "_C") -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"{name}{suffix}"


def build(force: bool = False, jobs: int = 0, debug: bool = False, verbose: bool = True, check: bool = False) -> Path:
    """check=True: the checked variant ``_C_check`` (device-side index validation with clamping and
    error words, PIO_CHECKS=1; host binding under UBSan), loaded instead of ``_C`` when
    ``PERCEIVER_CHECKED=1``."""
    bdir = BUILD / "check" if check else BUILD  # separate object caches per variant
    bdir.mkdir(parents=True, exist_ok=True)
    headers = sorted(HERE.glob("*.h"))
    hip_srcs = sorted(HERE.glob("*.hip"))
    opt = ["-O0", "-g"] if debug else ["-O3"]
    hip_flags = [f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=fast", "-munsafe-fp-atomics",
                 "-Wno-unused-result"] + opt + (["-DPIO_CHECKS=1"] if check else [])
    objs = []
    todo = []
    for src in hip_srcs:
        flags = hip_flags + PER_FILE_FLAGS.get(src.name, [])
        obj = bdir / f"{src.stem}.{_digest([src] + headers, flags)}.o"
        objs.append(obj)
        if force or not obj.exists():
            todo.append([HIPCC, *flags, "-I", str(HERE), "-c", str(src), "-o", str(obj)])
    inc, libdir = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    name = "_C_check" if check else "_C"
    san = ["-DPIO_CHECKS=1", "-fsanitize=undefined", "-fno-omit-frame-pointer"] if check else []
    cxx_flags = ["-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                 "-DTORCH_API_INCLUDE_EXTENSION_H", f"-DTORCH_EXTENSION_NAME={name}", "-D_GLIBCXX_USE_CXX11_ABI=1",
                 *san,
                 "-isystem", "/opt/rocm/include", "-isystem", py_inc] + sum((["-isystem", p] for p in inc), [])
    bsrc = HERE / "binding.cpp"
    # binding.cpp includes common.h (SlabJob, DropCfg, … are passed by value to the launchers):
    # its object must be rebuilt when a header changes, or the host and the kernels disagree on
    # a struct layout
    bobj = bdir / f"binding.{_digest([bsrc] + headers, cxx_flags)}.o"
    if force or not bobj.exists():
        todo.append(["g++", *cxx_flags, "-c", str(bsrc), "-o", str(bobj)])
    if todo:
        n = jobs or min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
        if verbose:
            print(f"[perceiver_io_amd] compiling {len(todo)} translation unit(s) for {ARCH} with {n} job(s)")
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(_run, todo))
    out = ext_path(name)
    # linked to a temporary name and renamed into place: a snapshot of the tree taken during a
    # build sees the previous or the new library, never a partly written one
    tmp = out.with_name(out.name + ".partial")
    link = ["g++", "-shared", *(["-fsanitize=undefined"] if check else []), "-o", str(tmp), str(bobj),
            *map(str, objs), f"-L{libdir}", "-L/opt/rocm/lib",
            "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lamdhip64", "-lc10_hip", "-ltorch_hip",
            f"-Wl,-rpath,{libdir}", "-Wl,-rpath,/opt/rocm/lib"]
    newest = max(p.stat().st_mtime for p in objs + [bobj])
    if force or todo or not out.exists() or out.stat().st_mtime < newest:
        _run(link)
        os.replace(tmp, out)
        if verbose:
            print(f"[perceiver_io_amd] linked {out.relative_to(PKG.parent)}")
    keep = {p.name for p in objs + [bobj]}
    for stale in bdir.glob("*.o"):  # objects of superseded sources (the cache holds the current ones)
        if stale.name not in keep:
            stale.unlink()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--check", action="store_true", help="build the checked variant _C_check")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, debug=a.debug, check=a.check)


if __name__ == "__main__":
    main()
