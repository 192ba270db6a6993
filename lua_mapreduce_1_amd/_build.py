"""In-tree build of the native parts of the framework.

* ``_lib/libmrhip.so`` — the CDNA4 (gfx950) HIP kernels in ``csrc/hip`` (wave64,
  LDS-tiled).  Built with ``hipcc --offload-arch=gfx950``; it links against the
  HIP runtime that torch already loaded (same soname ``libamdhip64.so.7``), so
  it must be loaded after ``import torch``.
* ``_lib/libmrcoord.so`` — the C++ coordinator (job table / control plane /
  blob store / persistent tables) in ``csrc/coord`` that replaces MongoDB
  (reference: mapreduce/cnn.lua, task.lua, persistent_table.lua, GridFS).
* ``_lib/libmrhost.so`` — native host-side input path: the multi-threaded
  split loader that reads split files straight into pinned memory
  (``csrc/host/loader.cpp``).

``*_stress.cpp`` files are test harnesses (built under sanitizers by
tests/test_native_sanitizers.py), not part of the libraries.

Everything is compiled in-tree so the ``.so`` files travel with the repository
snapshot to the GPU box (no JIT cache under ~/.cache).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(PKG, "_lib")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIP_LIB = os.path.join(LIBDIR, "libmrhip.so")
COORD_LIB = os.path.join(LIBDIR, "libmrcoord.so")
HOST_LIB = os.path.join(LIBDIR, "libmrhost.so")


def _newer(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {cmd[0]} (exit {r.returncode})")


def build_hip(force: bool = False, verbose: bool = False) -> str:
    srcdir = os.path.join(ROOT, "csrc", "hip")
    srcs = sorted(glob.glob(os.path.join(srcdir, "*.hip")))
    deps = srcs + sorted(glob.glob(os.path.join(srcdir, "*.h")))
    os.makedirs(LIBDIR, exist_ok=True)
    if not force and not _newer(HIP_LIB, deps):
        return HIP_LIB
    objs = []
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    headers = sorted(glob.glob(os.path.join(srcdir, "*.h")))
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not force and not _newer(o, [s] + headers):
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-Wno-unused-function", "-I", srcdir, "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    tmp = HIP_LIB + ".tmp"
    # libhsa-runtime64: the ROCr copy API of the SDMA downloads (csrc/hip/sdma.hip)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
         ["-L/opt/rocm/lib", "-lhsa-runtime64"])
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_cxx(name: str, srcsub: str, target: str, extra: list[str] | None = None,
              force: bool = False, verbose: bool = False) -> str:
    srcdir = os.path.join(ROOT, "csrc", srcsub)
    srcs = sorted(f for f in glob.glob(os.path.join(srcdir, "*.cpp")) if not f.endswith("_stress.cpp"))
    deps = srcs + sorted(glob.glob(os.path.join(srcdir, "*.h")))
    if not srcs:
        return ""
    os.makedirs(LIBDIR, exist_ok=True)
    if not force and not _newer(target, deps):
        return target
    tmp = target + ".tmp"
    cmd = ["g++", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wall", "-pthread", "-I", srcdir,
           "-o", tmp] + srcs + (extra or [])
    if verbose:
        print(" ".join(cmd))
    _run(cmd)
    os.replace(tmp, target)
    return target


def build_all(force: bool = False, verbose: bool = False) -> list[str]:
    out = [build_hip(force, verbose)]
    c = build_cxx("coord", "coord", COORD_LIB, force=force, verbose=verbose)
    if c:
        out.append(c)
    h = build_cxx("host", "host", HOST_LIB, force=force, verbose=verbose)
    if h:
        out.append(h)
    return out


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print("built", p)
