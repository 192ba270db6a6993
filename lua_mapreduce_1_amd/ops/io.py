"""Input staging: files / byte strings -> (pinned) host -> device tensors.

The bulk path is the native split loader (``csrc/host/loader.cpp``,
``_lib/libmrhost.so``): a pool of threads ``pread``s a rank's split files (or
byte ranges of one file) straight into the pinned staging buffer, publishing
a ready flag per split so the host->HBM copy of a chunk starts while later
splits are still being read.  The reference's map job reads its own split
file (examples/WordCount/mapfn.lua:4); here a rank reads only the splits it
owns, in parallel, without a bounce buffer.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time

import numpy as np
import torch

_HOST = None
_HOST_LOCK = threading.Lock()


def host_lib():
    """The native host library (built in-tree by ``_build.build_all``)."""
    global _HOST
    with _HOST_LOCK:
        if _HOST is None:
            from .. import _build
            if not os.path.exists(_build.HOST_LIB):
                _build.build_cxx("host", "host", _build.HOST_LIB)
            L = ctypes.CDLL(_build.HOST_LIB)
            P, I64 = ctypes.c_void_p, ctypes.c_int64
            L.mrh_load_start.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, ctypes.c_int, I64]
            L.mrh_load_start.restype = P
            L.mrh_load_done.argtypes = [P]
            L.mrh_load_done.restype = ctypes.c_int
            L.mrh_load_wait.argtypes = [P]
            L.mrh_load_wait.restype = ctypes.c_int
            L.mrh_drop_cache.argtypes = [ctypes.c_char_p]
            L.mrh_drop_cache.restype = ctypes.c_int
            _HOST = L
    return _HOST


class AsyncLoad:
    """Reads in flight: ``paths[i]`` bytes ``[file_off[i], file_off[i]+length[i])``
    land at ``dst[dst_off[i]:]`` (+ a ``\\n`` when ``pad[i]``); ``ready[i]`` turns
    1 when job i is complete.  ``dst`` must stay alive until :meth:`wait`."""

    def __init__(self, paths, file_off, length, dst_off, pad, dst: torch.Tensor, threads: int = 8,
                 piece: int = 8 << 20):
        n = len(paths)
        self.n = n
        self._keep = (dst, [p.encode() if isinstance(p, str) else p for p in paths])
        cpaths = (ctypes.c_char_p * max(n, 1))(*self._keep[1])
        self._arrs = [np.ascontiguousarray(a, dtype=np.int64) for a in (file_off, length, dst_off)]
        self._pad = np.ascontiguousarray(pad, dtype=np.int32)
        self.ready = np.zeros(max(n, 1), dtype=np.int32)
        self._cpaths = cpaths
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self._h = host_lib().mrh_load_start(n, ctypes.cast(cpaths, ctypes.c_void_p), *(ptr(a) for a in self._arrs),
                                            ptr(self._pad), ctypes.c_void_p(dst.data_ptr()), ptr(self.ready),
                                            int(threads), int(piece))
        if not self._h:
            raise RuntimeError("mrh_load_start failed")

    def done(self) -> int:
        return self.n if self._h is None else int(host_lib().mrh_load_done(self._h))

    def wait_jobs(self, j0: int, j1: int, poll: float = 20e-6) -> None:
        """Block until jobs [j0, j1) are complete (raises on a read error)."""
        r = self.ready
        while True:
            seg = r[j0:j1]
            if seg.min(initial=1) >= 1:
                return
            if (seg < 0).any():
                self.wait()
                raise OSError(f"split read failed (jobs {j0}..{j1})")
            time.sleep(poll)

    def wait(self) -> None:
        if self._h is not None:
            h, self._h = self._h, None
            rc = host_lib().mrh_load_wait(h)
            if rc != 0:
                raise OSError(-rc, os.strerror(-rc))

    def __del__(self):
        try:
            self.wait()
        except Exception:  # noqa: BLE001
            pass


def drop_page_cache(path: str) -> bool:
    """Evict a file's clean pages (posix_fadvise DONTNEED): the next read comes
    from the storage device (best effort; True when the call succeeded)."""
    return host_lib().mrh_drop_cache(path.encode()) == 0


def pinned_empty(nbytes: int) -> torch.Tensor:
    """Uninitialised uint8 host tensor in pinned memory of exactly ``nbytes``
    (csrc/hip/sort.hip mr_host_alloc).  torch's pinned allocator rounds a
    request up to a power of two, and pinning is paid per page: the 291 MB
    split buffer cost 22 ms as a 512 MB block (tools/cold_probe.py).  The
    memory is freed when the last tensor viewing it is gone."""
    import ctypes
    import weakref
    from . import _hip
    n = max(int(nbytes), 1)
    lib = _hip.lib()
    ptr = lib.mr_host_alloc(n)
    if not ptr:
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    arr = (ctypes.c_uint8 * n).from_address(ptr)
    f = weakref.finalize(arr, lib.mr_host_free, ptr)
    f.atexit = False  # at interpreter exit the process releases it (the HIP runtime may be gone)
    return torch.frombuffer(arr, dtype=torch.uint8)[:nbytes]


def read_file_bytes(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def bytes_to_device(data: bytes, device=None, pin: bool = True) -> torch.Tensor:
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.zeros(0, dtype=torch.uint8)
    if device is None or torch.device(device).type == "cpu":
        return t
    if pin:
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


def load_file(path: str, device=None) -> torch.Tensor:
    """Whole file as a uint8 tensor on ``device`` (host tensor when None/cpu),
    read by the native loader into (pinned) host memory first."""
    n = os.path.getsize(path)
    gpu = device is not None and torch.device(device).type != "cpu"
    host = torch.empty(n, dtype=torch.uint8, pin_memory=gpu)
    if n:
        AsyncLoad([path], [0], [n], [0], [0], host, threads=max(1, min(8, n >> 23))).wait()
    return host.to(device, non_blocking=True) if gpu else host
