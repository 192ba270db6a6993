"""Phase tracing: roctx ranges that show up on rocprofv3 timelines.

The reference has no tracer; it stores per-job wall/CPU times in the job
documents and aggregates them into the stats block (SURVEY.md §5.1,
task.lua:297, job.lua:127-147, server.lua:155-183, 555-600).  This framework
keeps those stats and adds named ranges around every phase of an iteration
(map launch, map wait, shuffle pack/exchange/all-to-all, reduce insert, tail,
finalize) and around worker jobs, through the ROCm tracing API (roctx, loaded
with ctypes; no Python dependency).  Ranges are off unless ``MR_ROCTX=1``:
then ``rocprofv3 --marker-trace`` (or ``--sys-trace``) records them.

    from lua_mapreduce_1_amd.utils import trace
    with trace.range("map"):
        ...
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

from .config import TUNABLES

_LIB = None
_ENABLED = TUNABLES.roctx
# host-only timeline without a profiler: MR_HOST_TIMELINE=1 records
# (name, start, end) perf_counter stamps of every range into LOG
LOG: list | None = [] if TUNABLES.host_timeline else None
_STACK: list = []
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


def _lib():
    global _LIB, _ENABLED
    if _LIB is None:
        for name in _CANDIDATES + tuple(os.path.join("/opt/rocm/lib", n) for n in _CANDIDATES):
            try:
                L = ctypes.CDLL(name)
            except OSError:
                continue
            L.roctxRangePushA.argtypes = [ctypes.c_char_p]
            L.roctxRangePushA.restype = ctypes.c_int
            L.roctxRangePop.argtypes = []
            L.roctxRangePop.restype = ctypes.c_int
            L.roctxMarkA.argtypes = [ctypes.c_char_p]
            L.roctxMarkA.restype = None
            _LIB = L
            break
        else:
            _ENABLED = False
            _LIB = False
    return _LIB


def enabled() -> bool:
    return _ENABLED and bool(_lib())


def enable(on: bool = True) -> bool:
    """Turn the ranges on/off at run time; returns whether roctx is available."""
    global _ENABLED
    _ENABLED = bool(on)
    return enabled()


def push(name: str) -> None:
    if LOG is not None:
        _STACK.append((name, time.perf_counter()))
    if _ENABLED and _lib():
        _LIB.roctxRangePushA(name.encode())


def pop() -> None:
    if LOG is not None and _STACK:
        name, t = _STACK.pop()
        LOG.append((name, t, time.perf_counter()))
    if _ENABLED and _LIB:
        _LIB.roctxRangePop()


def mark(name: str) -> None:
    if _ENABLED and _lib():
        _LIB.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx name
    if not _ENABLED and LOG is None:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()
