"""Worker -> GPU placement on a multi-GPU node (one worker process per GPU).

The reference's workers are single-threaded Lua processes with no device
(worker.lua); here a worker's map/reduce jobs run on a GPU, and N workers
started on one 8-GPU MI355X node must not all land on GPU 0 (they would
time-slice one device while seven idle). Each worker claims the lowest free
*slot* ``s`` with an exclusive ``flock`` on ``<dir>/lmr_gpu_slot.<s>`` and
uses device ``s % ndev``: the first ``ndev`` workers get one GPU each, later
ones wrap round. The lock lives as long as the worker's file descriptor, so a
worker that dies (even by SIGKILL) frees its slot for the next one, with no
coordinator round trip and nothing to clean up.

``HIP_VISIBLE_DEVICES`` still applies (``torch.cuda.device_count()`` counts
visible devices only, and does not initialise the GPU on this image).
"""
from __future__ import annotations

import fcntl
import os
import tempfile


class GpuSlot:
    """A claimed slot; ``device`` is the GPU index, ``release()`` frees it."""

    def __init__(self, slot: int, device: int, fd: int, path: str):
        self.slot, self.device, self._fd, self.path = slot, device, fd, path

    def release(self) -> None:
        if self._fd is not None:
            os.close(self._fd)  # closing the descriptor drops the flock
            self._fd = None

    def __del__(self):
        self.release()


def claim(ndev: int, lock_dir: str | None = None, max_slots: int = 4096) -> GpuSlot:
    """Claim the lowest free slot (non-blocking locks, so this never waits)."""
    if ndev < 1:
        raise ValueError("claim() needs at least one device")
    d = lock_dir or os.environ.get("MR_GPU_SLOT_DIR") or tempfile.gettempdir()
    os.makedirs(d, exist_ok=True)
    for s in range(max_slots):
        path = os.path.join(d, f"lmr_gpu_slot.{s}")
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o666)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            os.close(fd)
            continue
        return GpuSlot(s, s % ndev, fd, path)
    raise RuntimeError(f"no free GPU slot among {max_slots} in {d}")


def place_worker(gpu="auto") -> GpuSlot | int | None:
    """Select this worker's GPU before any GPU work: ``"auto"`` claims a slot
    when more than one device is visible, an int pins that device, ``None`` /
    ``"none"`` leaves torch's default. Returns the slot (keep it alive) or the
    pinned index."""
    if gpu is None or gpu == "none":
        return None
    import torch
    ndev = torch.cuda.device_count()
    if ndev < 1:
        return None
    if gpu == "auto":
        if ndev == 1:
            return None
        s = claim(ndev)
        torch.cuda.set_device(s.device)
        return s
    i = int(gpu)
    if not 0 <= i < ndev:
        raise ValueError(f"GPU {i} is not one of the {ndev} visible devices")
    torch.cuda.set_device(i)
    return i


def utest() -> None:
    with tempfile.TemporaryDirectory() as d:
        a, b, c = claim(2, d), claim(2, d), claim(2, d)
        assert (a.slot, b.slot, c.slot) == (0, 1, 2) and (a.device, b.device, c.device) == (0, 1, 0)
        b.release()
        e = claim(2, d)
        assert e.slot == 1 and e.device == 1
        for s in (a, c, e):
            s.release()
