"""Segmented operations over CSR value lists — the building blocks of batched
device reducers (``device_reducefn`` / ``device_combinerfn``, see
parallel/reducers.py).

A rank's keys and their value lists are one CSR pair: ``off`` (int64, m + 1
entries, ``off[0] == 0``, non-decreasing) and ``val`` (n values, int64 or
float64); key i's list is ``val[off[i]:off[i + 1]]``.  The reference hands
each list to the reducer one key at a time (/root/reference/mapreduce/
job.lua:264-284); these helpers fold ALL of a rank's lists at once:

* :func:`reduce` / :func:`sum` / :func:`min` / :func:`max` — one launch of
  ``mr_seg_reduce`` (csrc/hip/segments.hip: V values per thread, wave64
  segmented scan of the partial folds, one atomic per crossing segment and
  wavefront — skew-proof for hot keys), NumPy ``reduceat`` on CPU tensors;
* :func:`count`, :func:`mean`, :func:`first`, :func:`last`;
* :func:`sort` (values ordered inside each list: one stable radix sort by
  (segment, value)), :func:`unique`, :func:`nunique`, :func:`topk`,
  :func:`median`, :func:`quantile`;
* :func:`ids` (segment of every value), :func:`from_lengths`, :func:`take`
  (per-list slices).

Every function works on CUDA tensors (HIP kernels and device ops, no host
sync unless noted) and on CPU tensors (the executable specification).
"""
from __future__ import annotations

import builtins as _builtins

import numpy as np
import torch

from . import _hip

_I64_MAX, _I64_MIN = (1 << 63) - 1, -(1 << 63)
_OPS = {"sum": 0, "min": 1, "max": 2}


def _check(off: torch.Tensor, val: torch.Tensor) -> None:
    if off.dim() != 1 or off.numel() < 1:
        raise ValueError("off must be a 1-D int64 tensor of m + 1 offsets")
    if off.device != val.device:
        raise ValueError("off and val must be on the same device")


def lengths(off: torch.Tensor) -> torch.Tensor:
    """Number of values of each list (int64 [m])."""
    return off[1:] - off[:-1]


count = lengths


def from_lengths(lens: torch.Tensor) -> torch.Tensor:
    """CSR offsets (int64 [m + 1]) of lists of the given lengths."""
    out = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=lens.device)
    if lens.numel():
        torch.cumsum(lens.to(torch.int64), 0, out=out[1:])
    return out


def ids(off: torch.Tensor, n: int | None = None) -> torch.Tensor:
    """The list (segment) index of every value (int64 [n]).  ``n``: the
    number of values when the caller knows it (saves a host read)."""
    m = off.numel() - 1
    if n is None:
        n = int(off[-1])
    if m <= 0 or n == 0:
        return torch.zeros(n, dtype=torch.int64, device=off.device)
    return torch.repeat_interleave(torch.arange(m, dtype=torch.int64, device=off.device), lengths(off),
                                   output_size=n)


def _identity(dtype: torch.dtype, op: str):
    if op == "sum":
        return 0
    if dtype == torch.int64:
        return _I64_MAX if op == "min" else _I64_MIN
    return float("inf") if op == "min" else float("-inf")


def reduce(off: torch.Tensor, val: torch.Tensor, op: str = "sum", empty=None) -> torch.Tensor:
    """Fold of every list (``op``: sum | min | max); an empty list gives
    ``empty`` (default: the fold's identity — 0, or the dtype's max / min).
    int32 / float32 values fold as int64 / float64."""
    if op not in _OPS:
        raise ValueError(f"segment op {op!r}: one of {tuple(_OPS)}")
    _check(off, val)
    m = off.numel() - 1
    if val.dtype in (torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool):
        val = val.to(torch.int64)
    elif val.dtype in (torch.float32, torch.float16, torch.bfloat16):
        val = val.to(torch.float64)
    if val.dtype not in (torch.int64, torch.float64):
        raise TypeError(f"segment fold of {val.dtype} values")
    out = torch.full((m,), _identity(val.dtype, op), dtype=val.dtype, device=val.device)
    n = val.numel()
    if m and n:
        if val.is_cuda:
            off = off.to(torch.int64).contiguous()
            val = val.contiguous()
            _hip.call("mr_seg_reduce", _hip.ptr(off), m, _hip.ptr(val), n, 0 if val.dtype == torch.int64 else 1,
                      _OPS[op], _hip.ptr(out), _hip.stream(val.device))
        else:
            o = off.numpy().astype(np.int64)
            v = val.numpy()
            ln = np.diff(o)
            nz = np.flatnonzero(ln > 0)
            if nz.size:
                uf = {"sum": np.add, "min": np.minimum, "max": np.maximum}[op]
                out.numpy()[nz] = uf.reduceat(v, o[:-1][nz])
    if empty is not None and m:
        out = torch.where(lengths(off) > 0, out, torch.as_tensor(empty, dtype=out.dtype, device=out.device))
    return out


def sum(off, val):  # noqa: A001 - the fold's name
    return reduce(off, val, "sum")


def min(off, val, empty=None):  # noqa: A001
    return reduce(off, val, "min", empty)


def max(off, val, empty=None):  # noqa: A001
    return reduce(off, val, "max", empty)


def mean(off: torch.Tensor, val: torch.Tensor) -> torch.Tensor:
    """float64 mean of every list (NaN for an empty one)."""
    s = reduce(off, val.to(torch.float64) if not val.is_floating_point() else val, "sum")
    return s.to(torch.float64) / lengths(off).to(torch.float64)


def first(off: torch.Tensor, val: torch.Tensor, empty=0) -> torch.Tensor:
    ln = lengths(off)
    if val.numel() == 0:
        return torch.full((ln.numel(),), empty, dtype=val.dtype, device=val.device)
    g = val[off[:-1].clamp(max=val.numel() - 1)]
    return torch.where(ln > 0, g, torch.as_tensor(empty, dtype=val.dtype, device=val.device))


def last(off: torch.Tensor, val: torch.Tensor, empty=0) -> torch.Tensor:
    ln = lengths(off)
    if val.numel() == 0:
        return torch.full((ln.numel(),), empty, dtype=val.dtype, device=val.device)
    g = val[(off[1:] - 1).clamp(min=0)]
    return torch.where(ln > 0, g, torch.as_tensor(empty, dtype=val.dtype, device=val.device))


def order_key(val: torch.Tensor) -> torch.Tensor:
    """int64 whose UNSIGNED order is the numeric order of ``val`` (int64 or
    float64; -0.0 before +0.0, NaNs last) — the radix sort's key word."""
    sign = torch.tensor(_I64_MIN, dtype=torch.int64, device=val.device)
    if val.dtype == torch.float64:
        b = val.view(torch.int64)
        return torch.where(b < 0, ~b, b ^ sign)
    if val.dtype != torch.int64:
        val = val.to(torch.int64)
    return val ^ sign


def _bits(n: int) -> int:
    return _builtins.max(1, int(_builtins.max(n, 1) - 1).bit_length())


def sort_perm(off: torch.Tensor, val: torch.Tensor, descending: bool = False) -> torch.Tensor:
    """Permutation of ``val`` that orders every list's values (stable; lists
    stay in place)."""
    from .primitives import sort_keys_checked
    n = val.numel()
    m = off.numel() - 1
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=val.device)
    k = order_key(val)
    if descending:
        k = ~k
    return sort_keys_checked([ids(off, n), k], bits=[_bits(m), 64]).long()


def sort(off: torch.Tensor, val: torch.Tensor, descending: bool = False) -> torch.Tensor:
    """Every list's values in ascending (or descending) order (same ``off``)."""
    return val[sort_perm(off, val, descending)] if val.numel() else val.clone()


def take(off: torch.Tensor, val: torch.Tensor, start, stop) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-list slices ``val[off[i] + start[i] : off[i] + stop[i]]`` (start /
    stop: int or int64 [m], clamped to each list) -> (new off, new val)."""
    ln = lengths(off)
    m = ln.numel()
    d = off.device
    st = torch.as_tensor(start, dtype=torch.int64, device=d).expand(m).clamp(min=0)
    st = torch.minimum(st, ln)
    sp = torch.as_tensor(stop, dtype=torch.int64, device=d).expand(m)
    sp = torch.minimum(torch.maximum(sp, st), ln)
    nl = sp - st
    noff = from_lengths(nl)
    total = int(noff[-1]) if m else 0
    if total == 0:
        return noff, val[:0]
    seg = ids(noff, total)
    pos = torch.arange(total, dtype=torch.int64, device=d) - noff[seg] + off[seg] + st[seg]
    return noff, val[pos]


def unique(off: torch.Tensor, val: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Distinct values of every list, ascending -> (new off, new val)."""
    n = val.numel()
    m = off.numel() - 1
    if n == 0:
        return off.clone(), val.clone()
    p = sort_perm(off, val)
    sv = val[p]
    seg = ids(off, n)  # segments do not move: the sort keeps lists in place
    keep = torch.ones(n, dtype=torch.bool, device=val.device)
    keep[1:] = (seg[1:] != seg[:-1]) | (order_key(sv[1:]) != order_key(sv[:-1]))
    nl = torch.zeros(m, dtype=torch.int64, device=val.device)
    nl.index_add_(0, seg, keep.to(torch.int64))
    return from_lengths(nl), sv[keep]


def nunique(off: torch.Tensor, val: torch.Tensor) -> torch.Tensor:
    """Number of distinct values of every list (int64 [m])."""
    return lengths(unique(off, val)[0])


def topk(off: torch.Tensor, val: torch.Tensor, k: int, largest: bool = True) -> tuple[torch.Tensor, torch.Tensor]:
    """The k largest (or smallest) values of every list, in that order ->
    (new off, new val) (lists shorter than k keep all their values)."""
    return take(off, sort(off, val, descending=largest), 0, int(k))


def quantile(off: torch.Tensor, val: torch.Tensor, q: float) -> torch.Tensor:
    """Linear-interpolated q-quantile of every list (float64; NaN if empty)."""
    ln = lengths(off)
    sv = sort(off, val).to(torch.float64)
    if sv.numel() == 0:
        return torch.full((ln.numel(),), float("nan"), dtype=torch.float64, device=val.device)
    pos = (ln - 1).clamp(min=0).to(torch.float64) * float(q)
    lo = pos.floor().to(torch.int64)
    hi = pos.ceil().to(torch.int64)
    a = sv[(off[:-1] + lo).clamp(max=sv.numel() - 1)]
    b = sv[(off[:-1] + hi).clamp(max=sv.numel() - 1)]
    r = a + (b - a) * (pos - lo.to(torch.float64))
    return torch.where(ln > 0, r, torch.full_like(r, float("nan")))


def median(off: torch.Tensor, val: torch.Tensor) -> torch.Tensor:
    """Median of every list (float64: the mean of the two middle values of an
    even list; NaN if empty)."""
    return quantile(off, val, 0.5)
