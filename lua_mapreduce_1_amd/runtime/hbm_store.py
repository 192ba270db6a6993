"""Node-local intermediate files that stay in device memory ("hbm" storage).

The reference's storages all work across worker processes and hosts — GridFS
through mongod, ``shared`` through NFS, ``sshfs`` through scp
(/root/reference/mapreduce/fs.lua:185-208) — and a reduce job reads the map
files any worker wrote (job.lua:253-260).  ``hbm`` is the MI355X form of that
for the workers of ONE node:

* a map worker copies its partition files into an arena of device memory it
  owns (``hipMalloc`` chunks, exported with ``hipIpcGetMemHandle``);
* the coordinator's blob store keeps, under each file's name, a small
  descriptor (``MRH1`` + JSON: owner host/pid, chunk handle, offset, size,
  rows) instead of the bytes, so listing, counting and removing files work as
  with ``gridfs``;
* a reducer maps the owners' chunks (``hipIpcOpenMemHandle``, once per chunk)
  and pulls the files it needs with ONE gather-copy launch (over xGMI when
  the owner sits on another GPU) into one device buffer; a columnar fold's
  files are then decoded into the reduce table's input columns by ONE kernel
  (csrc/hip/ipc.hip) — the intermediate bytes never touch host memory or the
  coordinator socket;
* reduce results go to the coordinator like every storage's
  (job.lua:249-251: results always go to GridFS).

Without a GPU the arena chunks are files in ``/dev/shm`` (the same protocol
between host processes), so the storage is testable on a CPU-only machine.

Lifetime: an owner keeps its chunks until its worker starts the map phase of
a later iteration or finishes the task (every reduce of the iteration has then
read them).  A reducer on another host, or one whose owner process died,
cannot reach the files: the job fails like an ``sshfs`` job whose mapper host
is gone (fs.lua:141-181) and is retried / reported by the server.
"""
from __future__ import annotations

import ctypes
import json
import mmap
import os
import struct
import threading

import numpy as np

from .. import utils

MAGIC = b"MRH1"
CHUNK = 64 << 20  # arena chunk (a bigger file gets a chunk of its own)
ALIGN_MOD = 4     # files start at 4 mod 16: the 8-byte columns after MRC1's 20-byte header are aligned


def is_descriptor(b) -> bool:
    return bool(b) and bytes(b[:4]) == MAGIC


def _shm_dir() -> str:
    return os.environ.get("MR_HBM_SHM_DIR", "/dev/shm")


class _Chunk:
    __slots__ = ("cid", "size", "used", "ptr", "handle", "path", "mm")

    def __init__(self, cid: int, size: int):
        self.cid, self.size, self.used = cid, size, 0
        self.ptr = None      # device pointer (GPU arena)
        self.handle = b""    # hipIpcMemHandle_t bytes / shm file path
        self.path = None
        self.mm = None       # host mapping (CPU arena)


class HBMStore:
    """This process's arena (owner side) and its mapped peer chunks (reader
    side).  One per process; thread-safe (workers may be threads of one
    process)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._chunks: list[_Chunk] = []
        self._next = 0
        self._gen = None  # the (dbname, iteration) whose files the arena holds
        self._peers: dict = {}  # (host, pid, cid, handle) -> device ptr | mmap
        self.pid = os.getpid()
        self.host = utils.get_hostname()
        self._device = None
        self.stats = {"puts": 0, "put_bytes": 0, "pulls": 0, "pull_bytes": 0, "opened": 0}

    # -- owner side -----------------------------------------------------------
    def _gpu(self):
        if self._device is None:
            from . import device as dev
            self._device = dev.default_device()
        return self._device.type == "cuda"

    def _new_chunk(self, size: int) -> _Chunk:
        c = _Chunk(self._next, size)
        self._next += 1
        if not self._chunks and not getattr(self, "_atexit", False):
            import atexit
            atexit.register(self.release)  # (a /dev/shm chunk outlives its process otherwise)
            self._atexit = True
        if self._gpu():
            from ..ops import _hip
            p = ctypes.c_void_p()
            rc = _hip.lib().mr_ipc_alloc(size, ctypes.byref(p))
            if rc != 0 or not p.value:
                raise MemoryError(f"hbm storage: hipMalloc of {size} bytes failed ({rc})")
            h = ctypes.create_string_buffer(64)
            rc = _hip.lib().mr_ipc_handle(p, h)
            if rc != 0:
                _hip.lib().mr_ipc_free(p)
                raise RuntimeError(f"hbm storage: hipIpcGetMemHandle failed ({rc})")
            c.ptr, c.handle = p.value, h.raw
        else:
            c.path = os.path.join(_shm_dir(), f"lmr_hbm_{self.pid}_{c.cid}_{id(self)}")
            fd = os.open(c.path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
            try:
                os.ftruncate(fd, size)
                c.mm = mmap.mmap(fd, size)
            finally:
                os.close(fd)
            c.handle = c.path.encode()
        self._chunks.append(c)
        return c

    def _place(self, n: int) -> tuple[_Chunk, int]:
        for c in self._chunks[-1:]:
            off = (c.used + 15) // 16 * 16 + ALIGN_MOD
            if off + n <= c.size:
                c.used = off + n
                return c, off
        c = self._new_chunk(max(CHUNK, n + 32))
        c.used = ALIGN_MOD + n
        return c, ALIGN_MOD

    def put_many(self, items: list[tuple[str, bytes]], gen=None) -> list[tuple[str, bytes]]:
        """Copy the files into the arena; returns (name, descriptor) pairs for
        the coordinator.  ``gen`` = the task iteration the files belong to
        (the arena of an earlier one is released first)."""
        if not items:
            return []
        with self._lock:
            if gen is not None and self._gen is not None and gen != self._gen:
                self._release_locked()
            if gen is not None:
                self._gen = gen
            placed = [(name, data) + self._place(len(data)) for name, data in items]
            if self._gpu():
                self._upload(placed)
            else:
                for _name, data, c, off in placed:
                    c.mm[off:off + len(data)] = data
            out = []
            for name, data, c, off in placed:
                rows = struct.unpack_from("<Q", data, 4)[0] if data[:4] == b"MRC1" else -1
                d = {"host": self.host, "pid": self.pid, "dev": self._device.index if self._gpu() else -1,
                     "c": c.cid, "h": c.handle.hex(), "off": off, "len": len(data), "rows": rows}
                out.append((name, MAGIC + json.dumps(d, separators=(",", ":")).encode()))
                self.stats["puts"] += 1
                self.stats["put_bytes"] += len(data)
            return out

    def _upload(self, placed) -> None:
        """Host bytes -> their arena places: one pinned staging copy per
        chunk run, one H2D copy each (synchronous: the descriptors are
        published right after)."""
        import torch
        from ..ops import _hip
        by_chunk: dict = {}
        for _name, data, c, off in placed:
            by_chunk.setdefault(c.cid, (c, []))[1].append((off, data))
        for c, lst in by_chunk.values():
            lo = min(off for off, _ in lst)
            hi = max(off + len(d) for off, d in lst)
            stage = torch.empty(hi - lo, dtype=torch.uint8, pin_memory=True)
            a = stage.numpy()
            for off, d in lst:
                a[off - lo:off - lo + len(d)] = np.frombuffer(d, np.uint8)
            s = _hip.stream(self._device)
            _hip.call("mr_memcpy_async", ctypes.c_void_p(c.ptr + lo), _hip.ptr(stage), hi - lo, 1, s)
            torch.cuda.current_stream(self._device).synchronize()

    def release(self) -> None:
        """Free the arena (the files of the current iteration are consumed)
        and unmap every peer chunk."""
        with self._lock:
            self._release_locked()

    def _release_locked(self) -> None:
        if self._chunks and self._gpu():
            import torch
            torch.cuda.synchronize(self._device)  # (a copy may still read a chunk)
        for c in self._chunks:
            if c.ptr is not None:
                from ..ops import _hip
                _hip.lib().mr_ipc_free(ctypes.c_void_p(c.ptr))
            if c.mm is not None:
                c.mm.close()
            if c.path is not None:
                try:
                    os.unlink(c.path)
                except OSError:
                    pass
        self._chunks = []
        self._gen = None
        self._close_peers()

    def _close_peers(self) -> None:
        for v in self._peers.values():
            if isinstance(v, mmap.mmap):
                v.close()
            elif v is not None:
                from ..ops import _hip
                _hip.lib().mr_ipc_close(ctypes.c_void_p(v))
        self._peers = {}

    # -- reader side ------------------------------------------------------------
    @staticmethod
    def parse(desc: bytes) -> dict:
        if not is_descriptor(desc):
            raise ValueError("not an hbm file descriptor")
        return json.loads(bytes(desc[4:]))

    def _check_reachable(self, d: dict) -> None:
        if d["host"] != self.host:
            raise RuntimeError(f"hbm storage is node-local: a file of host {d['host']} is not reachable from "
                               f"{self.host} (use gridfs, shared or sshfs across hosts)")

    def _local_chunk(self, d: dict):
        if d["pid"] != self.pid:
            return None
        for c in self._chunks:
            if c.cid == d["c"] and c.handle.hex() == d["h"]:
                return c
        raise RuntimeError(f"hbm storage: chunk {d['c']} of this process is gone (file consumed twice?)")

    def _peer(self, d: dict):
        key = (d["host"], d["pid"], d["c"], d["h"])
        v = self._peers.get(key)
        if v is not None:
            return v
        h = bytes.fromhex(d["h"])
        if d["dev"] < 0:
            try:
                fd = os.open(h.decode(), os.O_RDONLY)
            except OSError as e:
                raise RuntimeError(f"hbm storage: the owner (pid {d['pid']}) of a map file is gone: {e}") from e
            try:
                v = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
            finally:
                os.close(fd)
        else:
            from ..ops import _hip
            p = ctypes.c_void_p()
            rc = _hip.lib().mr_ipc_open(ctypes.create_string_buffer(h, 64), ctypes.byref(p))
            if rc != 0 or not p.value:
                raise RuntimeError(f"hbm storage: hipIpcOpenMemHandle of a chunk of pid {d['pid']} on GPU {d['dev']} "
                                   f"failed ({rc}); is the owner still running?")
            v = p.value
        self._peers[key] = v
        self.stats["opened"] += 1
        return v

    def read_bytes(self, desc: bytes) -> bytes:
        """The file's bytes in host memory (host-plane reduces, the server)."""
        d = self.parse(desc)
        self._check_reachable(d)
        with self._lock:
            c = self._local_chunk(d)
            if c is not None and c.mm is not None:
                return bytes(c.mm[d["off"]:d["off"] + d["len"]])
            if c is None and d["dev"] < 0:
                mm = self._peer(d)
                return bytes(mm[d["off"]:d["off"] + d["len"]])
            src = c.ptr if c is not None else self._peer(d)
        import torch
        from ..ops import _hip
        out = torch.empty(d["len"], dtype=torch.uint8, pin_memory=True)
        dv = self._device if self._device is not None else torch.device("cuda", max(d["dev"], 0))
        _hip.call("mr_memcpy_async", _hip.ptr(out), ctypes.c_void_p(src + d["off"]), d["len"], 2, _hip.stream(dv))
        torch.cuda.current_stream(dv).synchronize()
        return out.numpy().tobytes()

    def read_many(self, descs: list[bytes]) -> list[bytes]:
        """Several files' bytes in host memory: on the GPU one gather-copy
        pull and ONE download, not a copy and a wait per file."""
        if not descs:
            return []
        if not self._gpu():
            return [self.read_bytes(x) for x in descs]
        buf, bases, ds = self.pull_device(descs, self._device)
        h = buf.cpu().numpy()
        return [h[b:b + d["len"]].tobytes() for b, d in zip(bases, ds)]

    def pull_device(self, descs: list[bytes], device):
        """The files into ONE device buffer, each at 4 mod 16 (ONE gather-copy
        launch; sources in this process's arena or peers' mapped chunks).
        -> (buf uint8 tensor, bases [int], descriptor dicts)."""
        import torch
        from ..ops import _hip
        ds = [self.parse(x) for x in descs]
        bases, total = [], 0
        for d in ds:
            self._check_reachable(d)
            off = (total + 15) // 16 * 16 + ALIGN_MOD
            bases.append(off)
            total = off + d["len"]
        buf = torch.empty(max(total, 16), dtype=torch.uint8, device=device)
        srcs = []
        with self._lock:
            self._gpu()
            for d in ds:
                c = self._local_chunk(d)
                srcs.append((c.ptr if c is not None else self._peer(d)) + d["off"])
        chunk = int(_hip.lib().mr_gather_copy_chunk())
        lens = np.array([d["len"] for d in ds], np.uint64)
        nch = (lens + np.uint64(chunk - 1)) // np.uint64(chunk)
        start = np.zeros(len(ds), np.uint64)
        if len(ds) > 1:
            np.cumsum(nch[:-1], out=start[1:])
        tab = np.concatenate([np.array(srcs, np.uint64), np.uint64(buf.data_ptr()) + np.array(bases, np.uint64),
                              lens, start])
        t = torch.from_numpy(tab.view(np.int64)).to(device)
        _hip.call("mr_gather_copy", _hip.ptr(t), len(ds), int(nch.sum()), _hip.stream(device))
        self.stats["pulls"] += len(ds)
        self.stats["pull_bytes"] += int(lens.sum())
        buf._mr_keep = t  # the copy table lives until the buffer does (stream order)
        return buf, bases, ds


_STORE: HBMStore | None = None
_STORE_LOCK = threading.Lock()


def store() -> HBMStore:
    global _STORE
    with _STORE_LOCK:
        if _STORE is None or _STORE.pid != os.getpid():
            _STORE = HBMStore()
        return _STORE


def release() -> None:
    """Free this process's arena and peer mappings (worker task end)."""
    if _STORE is not None and _STORE.pid == os.getpid():
        _STORE.release()
