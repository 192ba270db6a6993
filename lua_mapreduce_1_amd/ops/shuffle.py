"""Pack-by-destination for the all-to-all shuffle (HIP kernels in
``csrc/hip/shuffle.hip``; NumPy on CPU tensors).

``pack_by_dest`` lays a rank's distinct keys out as per-destination contiguous
record rows ``[hi, lo, val, loc]`` (loc = offset in the destination's key-byte
segment << 24 | length) plus the key bytes, and fills the count-exchange row
``[records, bytes, extra]`` per destination — three kernel launches, no sort,
no host synchronisation.  ``absolute_reps`` turns received locs into rep words
that index the received byte blob.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _hip
from . import keys as K
from .primitives import key_bytes_list


def pack_by_dest(hi, lo, val, rep, part, W: int, src, extra: int = 0, blob_capacity: int | None = None):
    """-> (rec int64 [n, 4], blob uint8, xchg int64 [3W]) (device or CPU)."""
    n = hi.numel()
    d = hi.device
    if hi.is_cuda:
        part = part.to(torch.int32).contiguous()
        cap = blob_capacity if blob_capacity is not None else (src.numel() if src is not None else 0) + 16 * n
        rec = torch.empty((n, 4), dtype=torch.int64, device=d)
        blob = torch.empty(max(cap, 1), dtype=torch.uint8, device=d)
        ws = torch.empty(6 * W, dtype=torch.int64, device=d)
        xchg = torch.empty(3 * W, dtype=torch.int64, device=d)
        _hip.call("mr_pack_by_dest", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(val), _hip.ptr(rep), _hip.ptr(part), n, W,
                  _hip.ptr(src) if src is not None else None, _hip.ptr(ws), _hip.ptr(xchg), int(extra),
                  _hip.ptr(rec), _hip.ptr(blob), 0, _hip.stream(d))
        return rec, blob, xchg
    dest = (part.numpy().astype(np.int64) % W)
    order = np.argsort(dest, kind="stable")
    kb = key_bytes_list(hi, lo, rep, src)
    lens = np.array([len(kb[i]) for i in order], dtype=np.int64)
    dsorted = dest[order]
    rec = np.empty((n, 4), dtype=np.int64)
    rec[:, 0] = hi.numpy()[order]
    rec[:, 1] = lo.numpy()[order]
    rec[:, 2] = val.numpy()[order]
    seg_start = np.zeros(W + 1, dtype=np.int64)
    np.add.at(seg_start, dsorted + 1, lens)
    seg_start = np.cumsum(seg_start)
    glob_off = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n else np.zeros(0, np.int64)
    loc_off = glob_off - seg_start[dsorted] if n else glob_off
    rec[:, 3] = (loc_off << K.REP_LEN_BITS) | np.minimum(lens, K.REP_LEN_MASK)
    blob = np.frombuffer(b"".join(kb[i] for i in order), dtype=np.uint8).copy() if n else np.zeros(0, np.uint8)
    counts = np.bincount(dest, minlength=W).astype(np.int64)
    xchg = np.stack([counts, seg_start[1:] - seg_start[:-1], np.full(W, extra, np.int64)], 1).reshape(-1)
    return torch.from_numpy(rec), torch.from_numpy(blob), torch.from_numpy(xchg)


def seg_bytes(rows: int, nbytes: int) -> int:
    """Bytes of one destination's segment in the combined layout."""
    return 32 * rows + ((nbytes + 7) & ~7)


STATUS_REDO = 1 << 40  # csrc/hip/shuffle.hip: added to the exchanged extra column by a rank that must redo its map


def pack_by_dest_combined(hi, lo, val, rep, part, W: int, src, extra: int = 0):
    """GPU: ONE uint8 buffer of per-destination segments [records (32 B:
    hi, lo, val, loc) | key bytes, padded to 8] + the count-exchange row
    [records, bytes, extra] per destination; destination d's segment is
    seg_bytes(rows_d, bytes_d) long, so the payload is a single all-to-all.
    -> (buf uint8, xchg int64 [3W])."""
    assert hi.is_cuda
    n = hi.numel()
    d = hi.device
    part = part.to(torch.int32).contiguous()
    cap = 32 * n + ((src.numel() if src is not None else 0) + 16 * n) + 8 * W
    ws, buf = _combined_bufs(d, W, cap)
    xchg = torch.empty(3 * W, dtype=torch.int64, device=d)
    _hip.call("mr_pack_by_dest", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(val), _hip.ptr(rep), _hip.ptr(part), n, W,
              _hip.ptr(src) if src is not None else None, _hip.ptr(ws), _hip.ptr(xchg), int(extra),
              _hip.ptr(buf), _hip.ptr(buf), 1, _hip.stream(d))
    return buf, xchg


def compact_pack(table, src, nparts: int, W: int, bound: int, extra: int = 0, errs=None, cap_bytes: int | None = None,
                 min_bytes: int = 0):
    """The W > 1 single-sync send side straight from the map's hash table
    (csrc/hip/shuffle.hip mr_compact_pack: three launches, no dense
    columns): every occupied slot -> its destination (FNV-1 partition of the
    key bytes, mod W) -> one uint8 buffer of per-destination segments
    [records (32 B) | key bytes], sized for ``bound`` rows; plus the
    count-exchange row and the table's key count on the device.  A rank
    whose table overflowed, whose chunk error words are set (``errs``) or
    whose segments outgrow the buffer adds STATUS_REDO to its exchanged
    extra column.  ``cap_bytes`` (tests): the buffer capacity the kernels
    assume, instead of the bound's.  ``min_bytes``: a floor on the capacity
    (the segment total a flagged exchange reported: keys that overlap in
    their source, e.g. n-gram spans, can need more key bytes than the
    bound-derived capacity holds).  -> (buf uint8, xchg int64 [3W], rows
    int64 [1])."""
    d = table.device
    lib = _hip.lib()
    cap = max(32 * bound + (src.numel() if src is not None else 0) + 16 * bound + 8 * W, int(min_bytes))
    ws, buf = _combined_bufs(d, W, cap)
    ncap = buf.numel() if cap_bytes is None else min(int(cap_bytes), buf.numel())
    nws = int(lib.mr_compact_pack_ws_bytes(table.cap, W))
    cw = _CP_WS.get(d)
    if cw is None or cw.numel() < nws:
        cw = _CP_WS[d] = torch.empty(nws + nws // 4, dtype=torch.uint8, device=d)
    xchg = torch.empty(3 * W, dtype=torch.int64, device=d)
    rows = torch.empty(1, dtype=torch.int64, device=d)
    e, ne = (_hip.ptr(errs), int(errs.numel())) if errs is not None and errs.numel() else (None, 0)
    _hip.call("mr_compact_pack", *table._gtab(), table.cap, nparts, W, _hip.ptr(src) if src is not None else None,
              _hip.ptr(cw), _hip.ptr(buf), ncap, _hip.ptr(xchg), int(extra), e, ne, _hip.ptr(rows),
              _hip.stream(d))
    return buf, xchg, rows


_CP_WS: dict = {}
_COMBINED: dict = {}


def _combined_bufs(d, W: int, cap: int):
    """Reused pack workspace and send buffer (grown as needed)."""
    ws, buf = _COMBINED.get(d, (None, None))
    if ws is None or ws.numel() < 6 * W:
        ws = torch.empty(6 * W, dtype=torch.int64, device=d)
    if buf is None or buf.numel() < cap:
        buf = torch.empty(cap + cap // 8, dtype=torch.uint8, device=d)
    _COMBINED[d] = (ws, buf)
    return ws, buf


def absolute_reps(rrec: torch.Tensor, recv_rows: list[int], recv_bytes: list[int]) -> torch.Tensor:
    """rep words (offset in the received blob << 24 | len) of received rows."""
    n = rrec.shape[0]
    W = len(recv_rows)
    rstart = np.concatenate([[0], np.cumsum(recv_rows)]).astype(np.int64)
    bstart = np.concatenate([[0], np.cumsum(recv_bytes)]).astype(np.int64)
    if rrec.is_cuda:
        d = rrec.device
        rs = torch.from_numpy(rstart).to(d, non_blocking=True)
        bs = torch.from_numpy(bstart).to(d, non_blocking=True)
        out = torch.empty(n, dtype=torch.int64, device=d)
        _hip.call("mr_fix_loc", _hip.ptr(rrec), n, _hip.ptr(rs), _hip.ptr(bs), W, _hip.ptr(out), _hip.stream(d))
        return out
    loc = rrec[:, 3].numpy().view(np.uint64)
    src_of = np.searchsorted(rstart, np.arange(n), side="right") - 1
    off = (loc >> np.uint64(K.REP_LEN_BITS)).astype(np.int64) + bstart[src_of]
    ln = (loc & np.uint64(K.REP_LEN_MASK)).astype(np.int64)
    return torch.from_numpy((off << K.REP_LEN_BITS) | ln)
