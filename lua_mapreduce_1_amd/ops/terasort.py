"""TeraSort record primitives (HIP kernels in ``csrc/hip/terasort.hip``; NumPy
on CPU tensors — the CPU path is the executable specification): the TeraGen
analogue and the checks of a sorted output (full keys, checksum, order).  The
sort itself is the record plane's (ops/records.py).

Records: 100 bytes = 10-byte key + 90-byte value, row-major uint8 tensors of
shape [n, 100].  Sort order: unsigned bytewise on the key = (hi, lo) with
hi = key bytes 0-7 big-endian and lo = key bytes 8-9 big-endian.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _hip

REC = 100
KEY = 10
M64 = (1 << 64) - 1


def _splitmix(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(M64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(M64)
    return x ^ (x >> np.uint64(31))


def generate(n: int, first: int, seed: int, device="cpu") -> torch.Tensor:
    """TeraGen analogue: records first .. first+n-1 of ``seed``."""
    d = torch.device(device)
    out = torch.empty((n, REC), dtype=torch.uint8, device=d)
    if d.type == "cuda":
        _hip.call("mr_ts_gen", _hip.ptr(out), n, first, seed, _hip.stream(d))
        return out
    with np.errstate(over="ignore"):
        r = np.arange(first, first + n, dtype=np.uint64)
        s = np.uint64(seed)
        k0 = _splitmix(s ^ (r * np.uint64(2)))
        k1 = _splitmix(s ^ (r * np.uint64(2) + np.uint64(1)))
        a = out.numpy()
        a[:, 0:8] = k0.astype(">u8").view(np.uint8).reshape(n, 8)
        a[:, 8:10] = k1.astype(">u8").view(np.uint8).reshape(n, 8)[:, 0:2]
        a[:, 10:18] = r.astype("<u8").view(np.uint8).reshape(n, 8)
        b = np.arange(18, REC, dtype=np.uint64)
        a[:, 18:] = (((r[:, None] * np.uint64(31) + b[None, :] * np.uint64(7)) & np.uint64(0x3F))
                     + np.uint64(0x30)).astype(np.uint8)
    return out


def keys(rec: torch.Tensor, ghist: torch.Tensor | None = None):
    """(hi, lo) int64 sort words of each record (validation: order checks).
    ``ghist`` (GPU, a zeroed int32 [2048]): also receives the digit
    histograms of hi's top 32 bits."""
    n = rec.shape[0]
    if rec.is_cuda:
        hi = torch.empty(n, dtype=torch.int64, device=rec.device)
        lo = torch.empty(n, dtype=torch.int64, device=rec.device)
        _hip.call("mr_ts_keys", _hip.ptr(rec), n, _hip.ptr(hi), _hip.ptr(lo),
                  _hip.ptr(ghist) if ghist is not None else None, _hip.stream(rec.device))
        return hi, lo
    a = rec.numpy()
    hi = np.ascontiguousarray(a[:, 0:8]).view(">u8").reshape(n).astype(np.uint64)
    lo = a[:, 8].astype(np.uint64) << np.uint64(8) | a[:, 9].astype(np.uint64)
    return torch.from_numpy(hi.view(np.int64)), torch.from_numpy(lo.view(np.int64))


def checksum(rec: torch.Tensor) -> int:
    """Order-independent 64-bit checksum of the records."""
    n = rec.shape[0]
    if rec.is_cuda:
        out = torch.zeros(1, dtype=torch.int64, device=rec.device)
        _hip.call("mr_ts_checksum", _hip.ptr(rec), n, _hip.ptr(out), _hip.stream(rec.device))
        return int(out.item()) & M64
    w = rec.numpy().view(np.uint32).reshape(n, REC // 4).astype(np.uint64)
    h = np.full(n, 0x243F6A8885A308D3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(REC // 4):
            x = h ^ w[:, j]
            x ^= x >> np.uint64(33)
            x *= np.uint64(0xFF51AFD7ED558CCD)
            x ^= x >> np.uint64(33)
            x *= np.uint64(0xC4CEB9FE1A85EC53)
            x ^= x >> np.uint64(33)
            h = x + np.uint64(j)
        return int(h.sum(dtype=np.uint64)) & M64


def unsorted_pairs(hi: torch.Tensor, lo: torch.Tensor) -> int:
    n = hi.numel()
    if hi.is_cuda:
        out = torch.zeros(1, dtype=torch.int64, device=hi.device)
        _hip.call("mr_ts_unsorted", _hip.ptr(hi), _hip.ptr(lo), n, _hip.ptr(out), _hip.stream(hi.device))
        return int(out.item())
    h = hi.numpy().view(np.uint64)
    lw = lo.numpy().view(np.uint64)
    return int(np.count_nonzero((h[:-1] > h[1:]) | ((h[:-1] == h[1:]) & (lw[:-1] > lw[1:]))))


