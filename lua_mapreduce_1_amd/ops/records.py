"""Fixed-width record primitives of the record plane (HIP kernels in
``csrc/hip/records.hip``; NumPy on CPU tensors — the executable
specification).  Rows are uint8 ``[n, rb]`` tensors keyed by their first
``kb`` bytes (1 <= kb <= 16, kb <= rb), ordered bytewise (unsigned,
big-endian) — TeraSort's 100-byte rows with 10-byte keys are one shape.

The sort is a radix sort of the 32-bit key prefixes (4 passes over u32 keys
and u32 row numbers) whose ties are ordered by the rest of the key read from
the rows; skewed keys (runs of more than 64 equal prefixes) fall back to a
sort of the full (hi, lo) key words.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _hip


def _check(rec: torch.Tensor, kb: int) -> tuple[int, int]:
    if rec.dim() != 2 or rec.dtype != torch.uint8:
        raise ValueError("records are a uint8 [n, row_bytes] tensor")
    rb = int(rec.shape[1])
    if not (1 <= kb <= 16 and kb <= rb):
        raise ValueError(f"key bytes must be 1..16 and at most the row width (got {kb} of {rb})")
    return int(rec.shape[0]), rb


def _host_keys(a: np.ndarray, kb: int) -> tuple[np.ndarray, np.ndarray]:
    n = a.shape[0]
    k = np.zeros((n, 16), np.uint8)
    k[:, :kb] = a[:, :kb]
    hi = np.ascontiguousarray(k[:, 0:8]).view(">u8").reshape(n).astype(np.uint64)
    lo = np.ascontiguousarray(k[:, 8:16]).view(">u8").reshape(n).astype(np.uint64)
    return hi, lo


def keys32(rec: torch.Tensor, kb: int, ghist: torch.Tensor | None = None) -> torch.Tensor:
    """Key bytes 0..3 big-endian (zero-padded) as the bit patterns of an
    int32 tensor.  ``ghist`` (GPU: a zeroed int32 [2048]) also receives their
    radix digit histograms ([8][256] layout, digits 0..3)."""
    n, rb = _check(rec, kb)
    if rec.is_cuda:
        out = torch.empty(n, dtype=torch.int32, device=rec.device)
        _hip.call("mr_rec_keys32", _hip.ptr(rec), n, rb, kb, _hip.ptr(out), _hip.ptr(ghist), _hip.stream(rec.device))
        return out
    hi, _ = _host_keys(rec.numpy(), kb)
    return torch.from_numpy((hi >> np.uint64(32)).astype(np.uint32).view(np.int32))


def keys(rec: torch.Tensor, kb: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(hi, lo) int64 key words: key bytes 0..7 and 8..15 big-endian, zero-padded."""
    n, rb = _check(rec, kb)
    if rec.is_cuda:
        hi = torch.empty(n, dtype=torch.int64, device=rec.device)
        lo = torch.empty(n, dtype=torch.int64, device=rec.device)
        _hip.call("mr_rec_keys", _hip.ptr(rec), n, rb, kb, _hip.ptr(hi), _hip.ptr(lo), _hip.stream(rec.device))
        return hi, lo
    hi, lo = _host_keys(rec.numpy(), kb)
    return torch.from_numpy(hi.view(np.int64)), torch.from_numpy(lo.view(np.int64))


_TIE_WS: dict = {}


def _tie_ws(d, words: int) -> torch.Tensor:
    """Scratch of the tie fix-up (a run counter, run starts, the scan's
    per-block run lists), per device."""
    w = _TIE_WS.get(d)
    if w is None or w.numel() < words:
        w = _TIE_WS[d] = torch.empty(words, dtype=torch.int64, device=d)
    return w


def sort(rec: torch.Tensor, kb: int, k32: torch.Tensor | None = None, ghist: torch.Tensor | None = None,
         defer: bool = False):
    """(permutation int32 (int64 on CPU), sorted 32-bit key prefixes) of the
    rows in key order (stable).  GPU: pass ``k32``/``ghist`` from
    :func:`keys32` to skip recomputing them.  ``defer``: no host sync — returns
    (perm, sk, bad) with ``bad`` a device int32[1], non-zero when the fast
    sort's order is invalid (a tie run too long for the fix-up, or a given-up
    look-back); the caller checks it later and then takes :func:`sort_full`."""
    from .primitives import sort_error, sort_error_word, sort_keys32
    n, rb = _check(rec, kb)
    if not rec.is_cuda:
        hi, lo = keys(rec, kb)
        from .primitives import sort_keys
        perm = sort_keys([hi, lo], bits=[64, 64])
        sk = keys32(rec, kb)[perm]
        return (perm, sk, torch.zeros(1, dtype=torch.int32)) if defer else (perm, sk)
    d = rec.device
    if k32 is None or ghist is None:
        ghist = torch.zeros(2048, dtype=torch.int32, device=d)
        k32 = keys32(rec, kb, ghist)
    perm, sk = sort_keys32(k32, ghist)
    bad = torch.zeros(1, dtype=torch.int32, device=d)
    cap = max(1024, n // 256)
    ws = _tie_ws(d, int(_hip.lib().mr_rec_tie_ws_words(n, cap)))
    _hip.call("mr_rec_tie_fixup", _hip.ptr(sk), _hip.ptr(perm), _hip.ptr(rec), n, rb, kb, _hip.ptr(bad),
              _hip.ptr(ws), cap, _hip.stream(d))
    if defer:
        err = sort_error_word(d)
        if err is not None:
            bad.bitwise_or_((err != 0).to(torch.int32) * 2)
        return perm, sk, bad
    if int(bad.item()) or sort_error(d):
        # skewed keys (a prefix shared by more than 64 rows), or a given-up
        # look-back: sort the full key words
        return sort_full(rec, kb, k32)
    return perm, sk


def sort_full(rec: torch.Tensor, kb: int, k32: torch.Tensor):
    """:func:`sort` by the full (hi, lo) key words (checked sort): the
    fallback when the prefix sort's fix-up cannot order the ties."""
    from .primitives import sort_keys_checked
    hi, lo = keys(rec, kb)
    perm = sort_keys_checked([hi, lo], bits=[64, 64])
    return perm, k32[perm.long()]


def gather(rec: torch.Tensor, perm: torch.Tensor, mode: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
    """rec[perm] (rows).  GPU: 16-byte LDS-staged row gather for rows of
    16-244 bytes (a multiple of 4; any row slice of a block), else the dword
    (or byte) gather; ``mode=1`` forces the dword gather (A/B probes, tests).
    ``out``: rows written there (contiguous [len(perm), row_bytes] uint8, e.g.
    a row slice of a larger block) instead of a new tensor.
    (A scatter through the inverse permutation lost: 16.6 vs 10.1 ms per
    10 GB, removed in round 5, profiles/r5/pruned/.)"""
    n = perm.numel()
    rb = int(rec.shape[1])
    if out is not None and (tuple(out.shape) != (n, rb) or out.dtype != torch.uint8 or not out.is_contiguous()
                            or out.device != rec.device):
        raise ValueError("gather: out must be a contiguous uint8 [len(perm), row_bytes] tensor on rec's device")
    if rec.is_cuda:
        if out is None:
            out = torch.empty((n, rb), dtype=torch.uint8, device=rec.device)
        if n == 0:
            return out
        if rec.shape[0] == 0:
            raise IndexError("gather from an empty record block")
        p = perm if perm.dtype == torch.int32 else perm.to(torch.int32)
        _hip.call("mr_rec_gather", _hip.ptr(rec), int(rec.shape[0]), _hip.ptr(p.contiguous()), n, rb, _hip.ptr(out),
                  int(mode), _hip.stream(rec.device))
        return out
    if out is not None:
        return torch.index_select(rec, 0, perm.long(), out=out)
    return rec[perm.long()]


def dest32(k32: torch.Tensor, splitters: torch.Tensor) -> torch.Tensor:
    """Range partition: number of splitters <= the 32-bit key prefix (int32;
    splitters: sorted unsigned 32-bit values as int32 bit patterns)."""
    n = k32.numel()
    if k32.is_cuda:
        out = torch.empty(n, dtype=torch.int32, device=k32.device)
        sp = splitters.to(device=k32.device, dtype=torch.int32).contiguous()
        _hip.call("mr_rec_dest32", _hip.ptr(k32), n, _hip.ptr(sp), sp.numel(), _hip.ptr(out),
                  _hip.stream(k32.device))
        return out
    h = k32.numpy().view(np.uint32)
    s = splitters.numpy().astype(np.int32).view(np.uint32)
    return torch.from_numpy(np.searchsorted(s, h, side="right").astype(np.int32))


def bucket32(k32: torch.Tensor, sub: torch.Tensor, K: int, W: int):
    """Exchange buckets of the record plane's range-pipelined exchange:
    sub-range a = number of sub-splitters <= the 32-bit key prefix
    (``sub``: R*K - 1 of them, R <= W), bucket (a % K) * W + a // K (round,
    then destination).  Returns (bucket int32, ghist): GPU — ghist is the
    int32 [2048] digit-histogram block of the buckets (digit 0 = rows per
    bucket; K * W <= 256), ready for ``sort_keys32(bucket, ghist, bits=8)``;
    CPU — ghist is None."""
    n = k32.numel()
    if k32.is_cuda and K * W <= 256 and sub.numel() <= 1023:
        out = torch.empty(n, dtype=torch.int32, device=k32.device)
        gh = torch.zeros(2048, dtype=torch.int32, device=k32.device)
        sp = sub.to(device=k32.device, dtype=torch.int32).contiguous()
        _hip.call("mr_rec_bucket32", _hip.ptr(k32), n, _hip.ptr(sp), sp.numel(), K, W, _hip.ptr(out), _hip.ptr(gh),
                  _hip.stream(k32.device))
        return out, gh
    a = dest32(k32, sub) if sub.numel() else torch.zeros(n, dtype=torch.int32, device=k32.device)
    return torch.remainder(a, K).mul_(W).add_(torch.div(a, K, rounding_mode="floor")), None


def hist32(k32: torch.Tensor) -> torch.Tensor:
    """GPU: the radix sort's digit histograms of 32-bit key prefixes (an int32
    [2048] block, digits 0..3 filled — the layout keys32(ghist=) gives) for
    prefixes that are already extracted."""
    gh = torch.zeros(2048, dtype=torch.int32, device=k32.device)
    _hip.call("mr_rec_hist32", _hip.ptr(k32), k32.numel(), _hip.ptr(gh), _hip.stream(k32.device))
    return gh


def sample32(k32: torch.Tensor, k: int, seed: int) -> torch.Tensor:
    """GPU: ``k`` 32-bit key prefixes (int64, unsigned values) of rows drawn
    with replacement by a counter-based hash of ``seed`` (-1s when there are
    no rows) — one launch."""
    out = torch.empty(k, dtype=torch.int64, device=k32.device)
    _hip.call("mr_rec_sample32", _hip.ptr(k32), k32.numel(), k, seed & 0xFFFFFFFFFFFFFFFF, _hip.ptr(out),
              _hip.stream(k32.device))
    return out


def pick_splitters(srt: torch.Tensor, R: int) -> torch.Tensor:
    """GPU: the R - 1 splitters (int32 bit patterns) at evenly spaced ranks of
    the non-negative entries of the sorted int64 sample ``srt`` (zeros when
    there are none) — one launch, no host round trip."""
    sp = torch.empty(max(R - 1, 0), dtype=torch.int32, device=srt.device)
    if R > 1:
        _hip.call("mr_rec_pick", _hip.ptr(srt), srt.numel(), R, _hip.ptr(sp), _hip.stream(srt.device))
    return sp


def xchg_rows(gh: torch.Tensor, K: int, W: int, failed: int, err: torch.Tensor | None):
    """GPU: the count-exchange rows [W][K+1] (int64: rows per round for each
    destination from the bucket histogram ``gh``, then ``failed``) and an
    int64[1] flag (the bucket sort's look-back gave up) — one launch."""
    xchg = torch.empty((W, K + 1), dtype=torch.int64, device=gh.device)
    flag = torch.empty(1, dtype=torch.int64, device=gh.device)
    _hip.call("mr_rec_xchg", _hip.ptr(gh), K, W, int(failed), _hip.ptr(err) if err is not None else None,
              _hip.ptr(xchg), _hip.ptr(flag), _hip.stream(gh.device))
    return xchg, flag


def unsorted_pairs(rec: torch.Tensor, kb: int) -> int:
    """Adjacent rows out of key order (0 for a sorted block)."""
    hi, lo = keys(rec, kb)
    if hi.numel() < 2:
        return 0
    if rec.is_cuda:
        sign = -(1 << 63)
        a, b = hi ^ sign, lo ^ sign
        bad = (a[:-1] > a[1:]) | ((a[:-1] == a[1:]) & (b[:-1] > b[1:]))
        return int(bad.sum())
    h, lw = hi.numpy().view(np.uint64), lo.numpy().view(np.uint64)
    return int(np.count_nonzero((h[:-1] > h[1:]) | ((h[:-1] == h[1:]) & (lw[:-1] > lw[1:]))))
