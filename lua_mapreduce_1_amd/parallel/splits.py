"""Host-side input stores of the SPMD engine: the page-cache analogue of the
reference's split files (/root/reference/mapreduce/examples/WordCountBig/
taskfn.lua:6-11 — one map job per file of ≤10k lines).

* :class:`SplitStore` — every split in ONE pinned buffer (in-memory splits,
  split files read by the native loader, or a blob of splits back to back),
  each followed by a newline unless it ends in one; a rank pins and reads
  only its contiguous byte-balanced share (:func:`assign_contiguous`);
* :class:`WindowedSplitStore` — split files read on demand into a ring of two
  pinned windows, for inputs larger than host memory.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils.config import TUNABLES


class SplitStore:
    """Host-resident input splits in ONE pinned buffer (the page-cache analogue
    of the reference's split files).  Every split is followed by a newline so
    tokens never straddle two splits.

    ``offsets`` are global (every split's padded size is known to every rank,
    for the byte-balanced job assignment); the buffer holds only the owned
    splits ``own = (i0, i1)`` — a rank pins and reads just its share
    (:meth:`from_files` / :meth:`from_blob` with ``rank, world``).  Those two
    fill the buffer asynchronously with the native loader (ops/io.py);
    :meth:`wait_ready` blocks until a range of splits has landed, so the
    engine's host->HBM copies start while later splits are still being read."""

    def __init__(self, splits: list[bytes] | None = None, pin: bool = True):
        splits = splits or []
        sizes = [len(s) + (0 if s[-1:] == b"\n" else 1) for s in splits]
        self._layout(sizes, (0, len(splits)), pin)
        view = self.buffer.numpy()
        for i, s in enumerate(splits):
            a = int(self.offsets[i])
            view[a:a + len(s)] = np.frombuffer(s, dtype=np.uint8)
            if sizes[i] > len(s):
                view[a + len(s)] = 10

    def _layout(self, sizes, own, pin: bool) -> None:
        self.offsets = np.zeros(len(sizes) + 1, dtype=np.int64)
        np.cumsum(np.asarray(sizes, dtype=np.int64), out=self.offsets[1:])
        self.own = (int(own[0]), int(own[1]))
        self.base = int(self.offsets[self.own[0]])
        nbytes = int(self.offsets[self.own[1]]) - self.base
        if pin and torch.cuda.is_available() and TUNABLES.pin_exact:
            from ..ops import io as mio
            self.buffer = mio.pinned_empty(nbytes)  # exact size: pinning is paid per page
        else:
            self.buffer = torch.empty(nbytes, dtype=torch.uint8, pin_memory=pin and torch.cuda.is_available())
        self._load = None
        self.paths = None

    @classmethod
    def _async(cls, paths, file_off, lens, pad, own, pin: bool, threads: int) -> "SplitStore":
        self = cls.__new__(cls)
        sizes = np.asarray(lens, dtype=np.int64) + np.asarray(pad, dtype=np.int64)
        self._layout(sizes, own, pin)
        i0, i1 = self.own
        if i1 > i0:
            from ..ops import io as mio
            dst_off = self.offsets[i0:i1] - self.base
            self._load = mio.AsyncLoad([paths[i] for i in range(i0, i1)], np.asarray(file_off)[i0:i1],
                                       np.asarray(lens)[i0:i1], dst_off, np.asarray(pad)[i0:i1], self.buffer,
                                       threads=threads)
        return self

    @classmethod
    def from_files(cls, paths: list[str], rank: int = 0, world: int = 1, pin: bool = True,
                   threads: int = 8) -> "SplitStore":
        """One split per file (the reference's split files, WordCountBig
        taskfn.lua:6-10).  Sizes come from stat; a file that does not end in
        a newline is followed by one (the same rule as the
        in-memory and blob stores, so line numbers agree); only this rank's
        contiguous byte-balanced share is read."""
        lens, pad = _file_pads(paths)
        own = assign_contiguous([n + p for n, p in zip(lens, pad)], rank, world)
        self = cls._async(list(paths), [0] * len(paths), lens, pad, own, pin, threads)
        self.paths = list(paths)
        return self

    @classmethod
    def from_blob(cls, path: str, offsets, rank: int = 0, world: int = 1, pin: bool = True,
                  threads: int = 8) -> "SplitStore":
        """Splits stored back to back in one file, split i at bytes
        ``[offsets[i], offsets[i+1])`` (the benchmark's corpus cache)."""
        offsets = np.asarray(offsets, dtype=np.int64)
        lens = offsets[1:] - offsets[:-1]
        mm = np.memmap(path, dtype=np.uint8, mode="r") if offsets[-1] else None
        last = [int(mm[o - 1]) if n else 0 for o, n in zip(offsets[1:], lens)] if mm is not None else []
        del mm
        pad = [0 if (n and b == 10) else 1 for n, b in zip(lens, last)]
        own = assign_contiguous((lens + np.asarray(pad, dtype=np.int64)).tolist(), rank, world)
        return cls._async([path] * len(lens), offsets[:-1], lens, pad, own, pin, threads)

    def __len__(self) -> int:
        return len(self.offsets) - 1

    def size(self, i: int) -> int:
        return int(self.offsets[i + 1] - self.offsets[i])

    def region(self, i0: int, i1: int) -> tuple[int, int]:
        """Byte range of splits [i0, i1) in :attr:`buffer` (owned splits only)."""
        if i0 < i1 and not (self.own[0] <= i0 and i1 <= self.own[1]):
            raise ValueError(f"splits [{i0}, {i1}) are not held by this store (own {self.own})")
        return int(self.offsets[i0]) - self.base, int(self.offsets[i1]) - self.base

    def all_ready(self) -> bool:
        return self._load is None or self._load.done() == self._load.n

    def wait_ready(self, i0: int, i1: int) -> None:
        """Block until splits [i0, i1) are in the buffer."""
        if self._load is not None and i1 > i0:
            self._load.wait_jobs(i0 - self.own[0], i1 - self.own[0])

    def finish_loading(self) -> None:
        if self._load is not None:
            self._load.wait()
            self._load = None

    def newline_counts(self, i0: int, i1: int) -> list[int]:
        """Newlines of each owned split [i0, i1) (its padding newline included)."""
        self.finish_loading()
        view = self.buffer.numpy() if self.buffer.device.type == "cpu" else self.buffer.cpu().numpy()
        out = []
        for i in range(i0, i1):
            a, b = self.region(i, i + 1)
            out.append(int(np.count_nonzero(view[a:b] == 10)))
        return out


class WindowedSplitStore(SplitStore):
    """Split files read on demand into a ring of two pinned windows (inputs
    larger than host memory): the engine's streaming rounds
    (``arena_cap_mb``) ask for one round of splits at a time
    (:meth:`load_round`), the native loader reads them into the free window,
    and the window is released once the round's host->HBM copies have
    completed.  Offsets/sizes of every split are known up front (stat)."""

    def __init__(self, paths: list[str], rank: int = 0, world: int = 1, window_mb: float = 256,
                 pin: bool = True, threads: int = 8):
        lens, pad = _file_pads(paths)
        self.paths = list(paths)
        self._lens, self._pad = lens, pad
        self.offsets = np.zeros(len(paths) + 1, dtype=np.int64)
        np.cumsum(np.asarray(lens, dtype=np.int64) + np.asarray(pad, dtype=np.int64), out=self.offsets[1:])
        self.own = assign_contiguous([n + p for n, p in zip(lens, pad)], rank, world)
        self.base = int(self.offsets[self.own[0]])
        self.window = int(window_mb * (1 << 20))
        self.threads = threads
        self._win = [torch.empty(self.window, dtype=torch.uint8, pin_memory=pin and torch.cuda.is_available())
                     for _ in range(2)]
        self._released = [None, None]
        self._load = None
        self.buffer = None  # no whole-share buffer: rounds only

    def all_ready(self) -> bool:
        return True

    def wait_ready(self, i0: int, i1: int) -> None:
        return None

    def load_round(self, i0: int, i1: int, slot: int) -> torch.Tensor:
        """Splits [i0, i1) (each followed by a newline) in window ``slot``;
        waits until the window's previous copies have completed."""
        ev = self._released[slot]
        if ev is not None:
            ev.synchronize()
        nbytes = int(self.offsets[i1] - self.offsets[i0])
        if nbytes > self.window:
            raise ValueError(f"round of {nbytes} bytes exceeds the {self.window}-byte host window")
        from ..ops import io as mio
        w = self._win[slot]
        ld = mio.AsyncLoad(self.paths[i0:i1], [0] * (i1 - i0), self._lens[i0:i1], self.offsets[i0:i1] - self.offsets[i0],
                           self._pad[i0:i1], w, threads=self.threads)
        ld.wait()
        return w[:nbytes]

    def release(self, slot: int, event) -> None:
        self._released[slot] = event

    def newline_counts(self, i0: int, i1: int) -> list[int]:
        """Newlines of each split [i0, i1) (its padding newline included),
        counted by reading the files in 16 MiB blocks."""
        out = []
        for i in range(i0, i1):
            n = 0
            with open(self.paths[i], "rb") as f:
                while True:
                    b = f.read(16 << 20)
                    if not b:
                        break
                    n += b.count(b"\n")
            out.append(n + int(self._pad[i]))
        return out


def _file_pads(paths) -> tuple[list[int], list[int]]:
    """(sizes, pads): pad 1 when a file's last byte is not a newline (then a
    newline follows the split: tokens never straddle splits, and the next
    split's first line gets its own global line number)."""
    lens, pad = [], []
    for p in paths:
        n = os.path.getsize(p)
        last = b""
        if n:
            with open(p, "rb") as f:
                f.seek(n - 1)
                last = f.read(1)
        lens.append(n)
        pad.append(0 if last == b"\n" else 1)
    return lens, pad


def assign_contiguous(weights, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [j0, j1) of items for ``rank``, balanced by weight."""
    n = len(weights)
    if world == 1:
        return 0, n
    c = np.concatenate([[0.0], np.cumsum(np.asarray(weights, dtype=np.float64))])
    tot = c[-1]
    cuts = [int(np.searchsorted(c, tot * r / world, side="left")) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, n
    return cuts[rank], max(cuts[rank], cuts[rank + 1])
