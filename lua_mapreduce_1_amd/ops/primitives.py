"""Device primitives of the MapReduce data plane.

Each function runs the gfx950 HIP kernel for CUDA(HIP) tensors and an
equivalent NumPy implementation for CPU tensors (tests / non-GPU workers).
u64 quantities are carried in ``torch.int64`` tensors (bit patterns), u32 in
``torch.int32``.

Kernel inventory -> function here:
  K1+K2+K3+K4+K5  wordcount_map (fused tokenize, exact key, LDS combine)
  K2+K3           tokenize
  K4 (generic)    HashTable.insert
  K6/K9           sort_keys (LSD radix sort, 8-bit digits, wave64 ballots)
  K7              bincount + sort by partition (pack)
  K8              reduce_by_key (segmented fold)
  K3 (partition)  key_meta (exact FNV-1 partition, key lengths)
  K10/K11         gather_key_bytes (materialise key bytes for output)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import keys as K
from . import _hip
from ..utils.config import TUNABLES

import os as _os

# "count" folds like "sum" (a map emits 1 per occurrence, the reduce side sums
# partial counts); "none": keys only (a vocabulary, or the general plane's
# key -> slot table: csrc/hip/generic.hip)
OPS = {"sum": 0, "min": 1, "max": 2, "count": 0, "none": 4}
# MR_DEBUG_CHECKS=1: validate the offsets/indices a kernel will dereference
# (with safe torch ops) before launching it, so a bad input raises in Python
# instead of faulting the GPU.
DEBUG_CHECKS = TUNABLES.debug_checks


def _check_reps(lo: torch.Tensor, rep: torch.Tensor, src, what: str) -> None:
    if not DEBUG_CHECKS or lo.numel() == 0:
        return
    is_long = (lo & 0xFF) == 0xFF
    if not bool(is_long.any()):
        return
    if src is None:
        raise RuntimeError(f"{what}: long keys but no byte source")
    r = rep[is_long]
    end = (r >> 24) + (r & ((1 << 24) - 1))
    if int(end.max()) > src.numel() or int(r.min()) < 0:
        raise RuntimeError(f"{what}: key bytes out of range (max end {int(end.max())} > {src.numel()})")
_I64_MAX = (1 << 63) - 1
_I64_MIN = -(1 << 63)


def _op_init(op: str) -> int:
    return {"sum": 0, "count": 0, "none": 0, "min": _I64_MAX, "max": _I64_MIN}[op]


def next_pow2(n: int) -> int:
    return 1 << max(0, (int(n) - 1).bit_length())


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


def _u64(t: torch.Tensor) -> np.ndarray:
    return _np(t).view(np.uint64)


def _t64(a: np.ndarray, device="cpu") -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(device)


# ---------------------------------------------------------------------------
_OVF_COUNTERS = 64
_OVF_ENTRIES = 1 << 18
_CTRL_SHARD0, _CTRL_STRIDE, _CTRL_SHARDS = 32, 32, 64  # csrc/hip/hashtab.h
_CTRL_WORDS = _CTRL_SHARD0 + _CTRL_STRIDE * _CTRL_SHARDS
_GHIST_RUNS = 0x100  # csrc/hip/sort.hip MR_GHIST_RUNS


class HashTable:
    """Open-addressing (128-bit key -> int64 value, rep) table.

    GPU: five HBM arrays + control words, filled by ``csrc/hip/hashtab.h``.
    CPU: pending arrays, reduced with ``np.unique`` at compaction.

    ``src``: the byte source every rep word of the table indexes (set by the
    owner: the map arena, the received shuffle buffer).  Long keys (>= 16
    bytes) that match on (prefix, 56-bit hash) are compared byte for byte
    through it, so colliding long keys are never merged (exact identity of the
    reference's string keys, job.lua:83-97).  Without a source a long key is
    identified by (prefix, hash) only.
    """

    def __init__(self, capacity: int, device="cpu", op: str = "sum", val_init: int | None = None):
        self.device = torch.device(device)
        self.op = op
        # the values' reset value (default: the op's identity)
        self.val_init = _op_init(op) if val_init is None else int(val_init)
        self.cap = next_pow2(max(1024, int(capacity)))
        self.src: torch.Tensor | None = None
        if self.device.type == "cuda":
            d = self.device
            # key records {tag, lo, hi, rep} (csrc/hip/hashtab.h GSlot: a probe
            # and its key compare touch one line); the four fields are strided
            # views of one [cap, 4] tensor; the values in their own array (the
            # folds' memory-side atomics off the probed lines)
            self.slots = torch.zeros((self.cap, 4), dtype=torch.int64, device=d)
            self.tag, self.lo, self.hi, self.rep = (self.slots[:, j] for j in range(4))
            self.val = torch.full((self.cap,), self.val_init, dtype=torch.int64, device=d)
            # [0] claims, [1] overflow flag, then 64 claim-count shards 128 B
            # apart (csrc/hip/hashtab.h CTRL_*): stats() sums them
            self.ctrl = torch.zeros(_CTRL_WORDS, dtype=torch.int32, device=d)
        else:
            self._pending: list[tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]] = []

    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def reset(self) -> None:
        self.src = None
        if self.is_cuda:
            _hip.call("mr_table_reset", _hip.ptr(self.slots), _hip.ptr(self.val), _hip.ptr(self.ctrl), self.cap,
                      self.val_init, _hip.stream(self.device))
            if getattr(self, "_ovf_counters", None) is not None and self._ovf_next:
                self._ovf_counters.zero_()
                self._ovf_next = 0
        else:
            self._pending = []

    def _gtab(self):
        """ctypes pointers (tag, hi, lo, val, rep, ctrl) of the table, as the
        native entry points take them: tag = the key records' base (the
        kernels read every record field from it), hi / lo / rep = the fields
        of record 0 (cached: the columns of a table never move)."""
        g = self.__dict__.get("_gtab_ptrs")
        if g is None or g[0] is not self.slots:
            b = self.slots.data_ptr()
            g = self._gtab_ptrs = (self.slots, (ctypes.c_void_p(b), ctypes.c_void_p(b + 16), ctypes.c_void_p(b + 8),
                                                _hip.ptr(self.val), ctypes.c_void_p(b + 24), _hip.ptr(self.ctrl)))
        return g[1]

    # -- inserts -------------------------------------------------------------
    def insert(self, hi: torch.Tensor, lo: torch.Tensor, val: torch.Tensor | None = None,
               rep: torch.Tensor | None = None, rep_add: int = 0, src: torch.Tensor | None = None) -> None:
        """Fold (key, value) rows in; rep words (+ ``rep_add``) index ``src``
        (default: the table's own source)."""
        n = hi.numel()
        if n == 0:
            return
        if src is not None:
            self.src = src
        if self.is_cuda:
            _hip.call("mr_hash_agg", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(val), _hip.ptr(rep), n, rep_add,
                      OPS[self.op], *self._gtab(), self.cap, _hip.ptr(self.src), _hip.stream(self.device))
        else:
            v = _np(val).astype(np.int64) if val is not None else np.ones(n, np.int64)
            r = _u64(rep).copy() if rep is not None else np.zeros(n, np.uint64)
            if rep is not None and rep_add:
                r = r + np.uint64(rep_add << K.REP_LEN_BITS)
            self._pending.append((_u64(hi).copy(), _u64(lo).copy(), v, r))

    def insert_spans(self, text: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor, val=None, rep_base: int = 0,
                     src: torch.Tensor | None = None) -> None:
        """Fold the keys ``text[starts[i] : starts[i] + lens[i]]`` (empty spans
        skipped) with values ``val`` (tensor, scalar, or None = 1); their rep
        words are ``rep_base + start`` in the table's byte source (the
        general plane's insert kernel, csrc/hip/generic.hip)."""
        n = starts.numel()
        if src is not None:
            self.src = src
        if n == 0:
            return
        if self.is_cuda:
            from . import agg as A
            a = A._ColsArg()
            a.k, a.list = 1, 0
            keep = []
            if isinstance(val, torch.Tensor):
                v = val.to(self.device)
                if v.dtype not in A._VT:
                    v = v.to(torch.float64 if v.is_floating_point() else torch.int64)
                v = v.contiguous()
                keep.append(v)
                a.src[0], a.stype[0] = v.data_ptr(), A._VT[v.dtype]
            else:
                a.stype[0], a.sbits[0] = A._VT_SCALAR, int(1 if val is None else val)
            a.dst[0], a.dtype[0], a.op[0] = self.val.data_ptr(), 0, OPS[self.op]
            st = starts.to(torch.int64).contiguous()
            ln = lens.to(torch.int32).contiguous()
            _hip.call("mr_agg_insert", *self._gtab(), self.cap, _hip.ptr(self.src), None, None, None, 0,
                      _hip.ptr(text), _hip.ptr(st), _hip.ptr(ln), rep_base, n, ctypes.byref(a),
                      _hip.stream(self.device))
            return
        buf = _np(text)
        st = _np(starts).astype(np.int64)
        ln = _np(lens).astype(np.int64)
        ok = (ln > 0) & (st >= 0)
        st, ln = st[ok], ln[ok]
        hi, lo = K.span_keys(buf, st, ln)
        rep = ((st.astype(np.uint64) + np.uint64(rep_base)) << np.uint64(K.REP_LEN_BITS)) | \
            np.minimum(ln, K.REP_LEN_MASK).astype(np.uint64)
        if isinstance(val, torch.Tensor):
            v = _np(val).astype(np.int64)[ok]
        else:
            v = np.full(st.size, 1 if val is None else int(val), np.int64)
        self._pending.append((hi, lo, v, rep))

    def _overflow(self, nbytes: int):
        """Overflow entries (hi, lo, rep) of the map kernel: tokens that found
        their workgroup's LDS table full (~10 per launch on the benchmark
        corpus).  Entries past the end are inserted into the HBM table
        directly, so the capacity only matters for speed: a fixed size (no
        re-allocation when a bigger launch comes along — a hipMalloc in the
        middle of an iteration cost ~5 ms)."""
        need = _OVF_ENTRIES
        if getattr(self, "_ovf", None) is None or self._ovf[0].numel() < need:
            d = self.device
            self._ovf = [torch.empty(need, dtype=torch.int64, device=d) for _ in range(3)]
            # one overflow counter per map launch between two resets (no fill
            # kernel in front of every chunk's map launch)
            self._ovf_counters = torch.zeros(_OVF_COUNTERS, dtype=torch.int64, device=d)
            self._ovf_next = 0
        if self._ovf_next == _OVF_COUNTERS:
            self._ovf_counters.zero_()
            self._ovf_next = 0
        self._ovf_counter = self._ovf_counters[self._ovf_next:self._ovf_next + 1]
        self._ovf_next += 1
        return self._ovf, self._ovf_counter

    def wordcount_map(self, text: torch.Tensor, rep_base: int = 0, src: torch.Tensor | None = None) -> None:
        """Fused tokenize + exact key + combine of every whitespace token
        (value 1): csrc/hip/wordcount3.hip.  ``text`` sits at byte
        ``rep_base`` of the table's byte source ``src`` (default: ``text``
        itself at 0)."""
        nbytes = text.numel()
        if src is not None:
            self.src = src
        elif self.src is None and rep_base == 0:
            self.src = text
        if nbytes == 0:
            return
        if self.is_cuda:
            assert text.dtype == torch.uint8 and text.is_contiguous()
            ovf, counter = self._overflow(nbytes)
            _hip.call("mr_wc_map3", _hip.ptr(text), nbytes, rep_base, *self._gtab(), self.cap,
                      _hip.ptr(ovf[0]), _hip.ptr(ovf[1]), _hip.ptr(ovf[2]), ovf[0].numel(), _hip.ptr(counter),
                      _hip.stream(self.device))
        else:
            buf = _np(text)
            starts, lens = K.token_spans(buf)
            hi, lo = K.span_keys(buf, starts, lens)
            rep = ((starts.astype(np.uint64) + np.uint64(rep_base)) << np.uint64(K.REP_LEN_BITS)) | \
                np.minimum(lens, K.REP_LEN_MASK).astype(np.uint64)
            self._pending.append((hi, lo, np.ones(hi.size, np.int64), rep))

    def insert_received(self, rec: torch.Tensor, recv_counts: torch.Tensor, W: int, rows: int | None = None,
                        src: torch.Tensor | None = None) -> None:
        """Fold all-to-all-received records into the table; ``recv_counts`` =
        the device count-exchange row [W, 3] (rows, key bytes, extra) per
        source.  ``rec``: int64 [n, 4] records (hi, lo, val, loc) whose key
        bytes were received separately (rep words become offsets into the
        concatenated received bytes), or — with ``rows`` = n — the uint8
        buffer of the combined layout (ops/shuffle.pack_by_dest_combined),
        whose rep words then index that same buffer.  One launch."""
        combined = rows is not None
        n = rows if combined else rec.shape[0]
        self.src = rec if combined else src
        if n == 0:
            return
        if self.is_cuda:
            assert rec.is_contiguous() and recv_counts.is_contiguous()
            _hip.call("mr_insert_received", _hip.ptr(rec), n, _hip.ptr(recv_counts), W, *self._gtab(), self.cap,
                      OPS[self.op], 1 if combined else 0, _hip.ptr(self.src), _hip.stream(self.device))
            return
        assert not combined, "the combined layout is GPU-only"
        from .shuffle import absolute_reps
        rc = recv_counts.view(W, 3).tolist()
        rep = absolute_reps(rec, [r[0] for r in rc], [r[1] for r in rc])
        self.insert(rec[:, 0].contiguous(), rec[:, 1].contiguous(), rec[:, 2].contiguous(), rep)

    def rehome_long_keys(self, buf: torch.Tensor, lo_off: int, hi_off: int, heap: torch.Tensor,
                         heap_cap: int) -> None:
        """Copy the bytes of long keys whose rep points into buf[lo_off:hi_off)
        to the key heap at the front of ``buf`` (``heap`` = int64[2] bump
        counter + full flag) and re-point their reps (streaming map rounds)."""
        if self.is_cuda:
            _hip.call("mr_table_rehome", _hip.ptr(self.slots), self.cap, _hip.ptr(buf), lo_off, hi_off,
                      _hip.ptr(heap), heap_cap, _hip.stream(self.device))
            return
        b = _np(buf) if not buf.is_cuda else None
        h = heap.numpy()
        for k, (hi_, lo_, v, r) in enumerate(self._pending):
            long_ = (lo_ & np.uint64(0xFF)) == np.uint64(K.LONG_MARK)
            off = r >> np.uint64(K.REP_LEN_BITS)
            sel = np.flatnonzero(long_ & (off >= np.uint64(lo_off)) & (off < np.uint64(hi_off)))
            for i in sel:
                o, n = int(r[i]) >> K.REP_LEN_BITS, int(r[i]) & K.REP_LEN_MASK
                d = int(h[0])
                if d + n > heap_cap:
                    h[1] = 1
                    continue
                b[d:d + n] = b[o:o + n].copy()
                h[0] = d + n
                r[i] = np.uint64(K.make_rep(d, n))

    # -- state ---------------------------------------------------------------
    def stats(self) -> tuple[int, bool]:
        """(occupied slots, overflowed).  Synchronises on GPU."""
        if self.is_cuda:
            c = host_read(self.ctrl)
            return int(c[0]) + int(c[_CTRL_SHARD0::_CTRL_STRIDE].sum()), bool(c[1])
        return sum(p[0].size for p in self._pending), False

    def compact(self, known_stats: tuple[int, bool] | None = None, aos: bool = False):
        """Dense (hi, lo, val, rep) of all occupied slots (slot order on GPU).
        ``known_stats``: the (n, overflow) of a stats() call made since the last
        insert (saves a second host synchronisation).  ``aos``: also the rows
        as int64 [n, 4] records for :func:`gather_aos4` (a fifth value; None
        on CPU)."""
        if self.is_cuda:
            n, ovf = known_stats if known_stats is not None else self.stats()
            if ovf:
                raise OverflowError("hash table overflow")
            d = self.device
            out = [torch.empty(n, dtype=torch.int64, device=d) for _ in range(4)]
            rec = torch.empty((n, 4), dtype=torch.int64, device=d) if aos else None
            counter = torch.zeros(1, dtype=torch.int64, device=d)
            _hip.call("mr_table_compact", *self._gtab(), self.cap, *[_hip.ptr(o) for o in out],
                      _hip.ptr(counter), _hip.ptr(rec), _hip.stream(d))
            return tuple(out) + ((rec,) if aos else ())
        if not self._pending:
            z = torch.zeros(0, dtype=torch.int64)
            return (z, z.clone(), z.clone(), z.clone()) + ((None,) if aos else ())
        hi = np.concatenate([p[0] for p in self._pending])
        lo = np.concatenate([p[1] for p in self._pending])
        v = np.concatenate([p[2] for p in self._pending])
        r = np.concatenate([p[3] for p in self._pending])
        keys = np.empty(hi.size, dtype=[("hi", np.uint64), ("lo", np.uint64), ("d", np.int64)])
        keys["hi"], keys["lo"], keys["d"] = hi, lo, 0
        long_ = (lo & np.uint64(0xFF)) == np.uint64(K.LONG_MARK)
        if long_.any() and self.src is not None:
            # exact identity of long keys: equal (prefix, hash) but different
            # bytes get different ids (the device tables compare bytes)
            sb = _np(self.src)
            ids: dict = {}
            d = keys["d"]
            for i in np.flatnonzero(long_):
                rr = int(r[i])
                o, ln = rr >> K.REP_LEN_BITS, rr & K.REP_LEN_MASK
                d[i] = ids.setdefault(sb[o:o + ln].tobytes(), len(ids) + 1)
        uk, first, inv = np.unique(keys, return_index=True, return_inverse=True)
        if self.op in ("sum", "count", "none"):
            agg = np.zeros(uk.size, np.int64)
            np.add.at(agg, inv, v)
        elif self.op == "min":
            agg = np.full(uk.size, _I64_MAX, np.int64)
            np.minimum.at(agg, inv, v)
        else:
            agg = np.full(uk.size, _I64_MIN, np.int64)
            np.maximum.at(agg, inv, v)
        return (_t64(uk["hi"].copy()), _t64(uk["lo"].copy()), torch.from_numpy(agg), _t64(r[first])) + \
            ((None,) if aos else ())


def gather_aos4(perm: torch.Tensor, aos: torch.Tensor, want_len: bool = False):
    """(hi, lo, val, rep) of the 32-byte records ``aos[perm]`` (GPU: one
    launch, one 32-byte record read per row instead of one line per column)
    — and, with ``want_len``, the gathered keys' lengths as a fifth column
    (key_meta's lengths, from the same launch)."""
    n = perm.numel()
    d = aos.device
    out = [torch.empty(n, dtype=torch.int64, device=d) for _ in range(5 if want_len else 4)]
    if n:
        _hip.call("mr_gather_aos4", _hip.ptr(perm.to(torch.int32).contiguous()), n, _hip.ptr(aos),
                  *[_hip.ptr(o) for o in out[:4]], _hip.ptr(out[4]) if want_len else None, _hip.stream(d))
    return tuple(out)


# ---------------------------------------------------------------------------
def tokenize(text: torch.Tensor, rep_base: int = 0, chunk_bytes: int = 64 * 1024):
    """Per-token (hi, lo, rep) in text order on CPU, arbitrary order on GPU."""
    nbytes = text.numel()
    if text.is_cuda:
        d = text.device
        counter = torch.zeros(1, dtype=torch.int64, device=d)
        _hip.call("mr_count_tokens", _hip.ptr(text), nbytes, chunk_bytes, _hip.ptr(counter), _hip.stream(d))
        n = int(counter.item())
        out = [torch.empty(n, dtype=torch.int64, device=d) for _ in range(3)]
        counter.zero_()
        _hip.call("mr_tokenize", _hip.ptr(text), nbytes, chunk_bytes, rep_base, *[_hip.ptr(o) for o in out], n,
                  _hip.ptr(counter), _hip.stream(d))
        return tuple(out)
    buf = _np(text)
    starts, lens = K.token_spans(buf)
    hi, lo = K.span_keys(buf, starts, lens)
    rep = ((starts.astype(np.uint64) + np.uint64(rep_base)) << np.uint64(K.REP_LEN_BITS)) | \
        np.minimum(lens, K.REP_LEN_MASK).astype(np.uint64)
    return _t64(hi), _t64(lo), _t64(rep)


def key_meta(hi: torch.Tensor, lo: torch.Tensor, rep: torch.Tensor, src: torch.Tensor | None,
             nparts: int = 0, want_part: bool = True, want_len: bool = True, want_w1: bool = False,
             want_k7: bool = False):
    """(partition id int32 | None, key length int64 | None).

    Partition = exact uint32 FNV-1 of the key bytes mod ``nparts`` (raw hash
    when nparts == 0).  Long-key bytes are read from ``src`` at rep offsets.
    ``want_w1`` (with ``want_part``): a third value, ``key_word(..., 1)``
    computed in the same pass over the key bytes.  ``want_k7`` (GPU, with
    ``want_w1``, 1 <= nparts <= 256): a fourth, ``(k7, bad)`` — the two words
    of the 15-pass sort of 7-bit keys (``k7[0]`` = partition << 56 | bytes
    0-7 as 7-bit digits, ``k7[1]`` = bytes 8-15 likewise) and a device int32
    flag, nonzero when some key has a byte >= 0x80 in its first 16 (k7's
    order is then not the key order).
    """
    n = hi.numel()
    if hi.is_cuda:
        _check_reps(lo, rep, src, "key_meta")
        d = hi.device
        part = torch.empty(n, dtype=torch.int32, device=d) if want_part else None
        ln = torch.empty(n, dtype=torch.int64, device=d) if want_len else None
        w1 = torch.empty(n, dtype=torch.int64, device=d) if (want_w1 and want_part) else None
        k7 = bad = alpha = None
        if want_k7 and w1 is not None and 1 <= nparts <= 256:
            k7 = torch.empty((2, n), dtype=torch.int64, device=d)
            bad = torch.zeros(1, dtype=torch.int32, device=d)
            if TUNABLES.exact_alpha:
                alpha = torch.zeros(4, dtype=torch.int32, device=d)
        srcp = _hip.ptr(src) if src is not None else None
        _hip.call("mr_key_meta", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep), n, srcp, nparts, _hip.ptr(part),
                  _hip.ptr(ln), _hip.ptr(w1), _hip.ptr(k7), _hip.ptr(bad), _hip.ptr(alpha), _hip.stream(d))
        if want_k7:
            return part, ln, w1, (None if k7 is None else (k7, bad, alpha))
        return (part, ln, w1) if want_w1 else (part, ln)
    b = key_bytes_list(hi, lo, rep, src)
    part = None
    if want_part:
        h = np.array([K.fnv1(x) for x in b], dtype=np.uint64)
        part = torch.from_numpy((h % np.uint64(nparts) if nparts else h).astype(np.uint32).view(np.int32))
    ln = torch.tensor([len(x) for x in b], dtype=torch.int64) if want_len else None
    if want_w1 or want_k7:
        w1 = key_word(hi, lo, rep, src, 1) if want_part else None
        return (part, ln, w1, None) if want_k7 else (part, ln, w1)
    return part, ln


def key_bytes_list(hi, lo, rep, src) -> list[bytes]:
    """Host list of key byte strings (CPU helper; also used after D2H)."""
    h = _u64(hi)
    lw = _u64(lo)
    r = _u64(rep) if rep is not None else None
    s = _np(src) if src is not None else None
    out = []
    for i in range(h.size):
        l_ = int(lw[i])
        if (l_ & 0xFF) != K.LONG_MARK:
            out.append(K.unpack_key(int(h[i]), l_))
        else:
            rr = int(r[i])
            off, ln = rr >> K.REP_LEN_BITS, rr & K.REP_LEN_MASK
            out.append(bytes(s[off:off + ln]))
    return out


def exclusive_scan(x: torch.Tensor):
    """Exclusive prefix sum of an int32/int64 tensor -> (out, total)."""
    n = x.numel()
    if x.is_cuda:
        d = x.device
        out = torch.empty_like(x)
        lib = _hip.lib()
        parts = torch.empty(int(lib.mr_scan_partials_len(max(n, 1))), dtype=x.dtype, device=d)
        total = torch.zeros(1, dtype=x.dtype, device=d)
        name = "mr_exclusive_scan_u32" if x.dtype == torch.int32 else "mr_exclusive_scan_i64"
        _hip.call(name, _hip.ptr(x), _hip.ptr(out), n, _hip.ptr(parts), _hip.ptr(total), _hip.stream(d))
        return out, total
    c = torch.cumsum(x, 0)
    tot = c[-1:].clone() if n else torch.zeros(1, dtype=x.dtype)
    return (c - x).to(x.dtype), tot


def gather_key_bytes(hi, lo, rep, src, lengths: torch.Tensor | None = None, capacity: int | None = None):
    """Materialise key bytes: (offsets int64[n+1], blob uint8).

    With ``capacity`` (GPU) the blob is allocated at that size and NOT trimmed,
    so no host synchronisation is needed; the used size is ``offsets[-1]``
    (a device value).  Any bound >= the total works, e.g. the byte size of the
    text the keys came from (distinct keys occupy disjoint occurrences).
    """
    n = hi.numel()
    if lengths is None:
        _, lengths = key_meta(hi, lo, rep, src, want_part=False)
    off, total = exclusive_scan(lengths)
    if hi.is_cuda:
        _check_reps(lo, rep, src, "gather_key_bytes")
        if DEBUG_CHECKS and capacity is not None and int(total.item()) > capacity:
            raise RuntimeError(f"gather_key_bytes: {int(total.item())} bytes > capacity {capacity}")
        d = hi.device
        nb = int(total.item()) if capacity is None else int(capacity)
        blob = torch.empty(max(nb, 1), dtype=torch.uint8, device=d)
        srcp = _hip.ptr(src) if src is not None else None
        _hip.call("mr_gather_key_bytes", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep), _hip.ptr(off), n, srcp,
                  _hip.ptr(blob), blob.numel(), _hip.stream(d))
        if capacity is None:
            blob = blob[:nb]
        return torch.cat([off, total]), blob
    b = key_bytes_list(hi, lo, rep, src)
    blob = torch.frombuffer(bytearray(b"".join(b)), dtype=torch.uint8) if b else torch.zeros(0, dtype=torch.uint8)
    return torch.cat([off, total]), blob


_HOST_READ: dict = {}


def host_read(t: torch.Tensor) -> np.ndarray:
    """Small device tensor -> host numpy copy: download on the current stream
    (mr_d2h_async: shader stores into a reused pinned buffer, so it does not
    wait behind input copies queued on the shared SDMA engine, as ``.cpu()``
    does), then wait for the current stream only."""
    if not t.is_cuda:
        return t.detach().numpy().copy()
    t = t.contiguous()
    nb = t.numel() * t.element_size()
    buf = _HOST_READ.get(t.device)
    if buf is None or buf.numel() < nb:
        buf = torch.empty(max(nb, 1 << 12), dtype=torch.uint8, pin_memory=True)
        _HOST_READ[t.device] = buf
    _hip.call("mr_d2h_async", _hip.ptr(buf), _hip.ptr(t), nb, _hip.stream(t.device))
    _hip.wait_stream(t.device)
    return buf[:nb].numpy().view(_NP_DTYPE[t.dtype]).reshape(tuple(t.shape)).copy()


class HostRead:
    """Small device tensors queued for download (host_read_begin); wait()
    returns their host copies.  Up to 8 tensors of <= 16 KiB in total go in
    one launch that also signals the host (mr_small_d2h); the host work done
    between begin and wait overlaps the download."""

    def __init__(self, ts: list):
        self.ts = [t.contiguous() for t in ts]
        self.views = None
        self.sig = None
        if not self.ts or not self.ts[0].is_cuda:
            return
        d = self.ts[0].device
        self.device = d
        sizes = [t.numel() * t.element_size() for t in self.ts]
        total = sum((n + 15) & ~15 for n in sizes)
        if len(self.ts) > 8 or total > _SMALL_SLOT or _hip.SPIN_S <= 0:
            return  # host_read_many's blits + wait
        ring = _SMALL_READ.get(d)
        if ring is None:
            p = _hip.lib().mr_host_alloc(_SMALL_SLOT * _SMALL_SLOTS)
            if not p:
                raise RuntimeError("hipHostMalloc of the small-download buffer failed")
            ring = _SMALL_READ[d] = [p, np.ctypeslib.as_array((ctypes.c_uint8 * (_SMALL_SLOT * _SMALL_SLOTS)).from_address(p)),
                                     0]
        # a ring of slots: up to _SMALL_SLOTS reads may be outstanding at once
        k = ring[2]
        ring[2] = (k + 1) % _SMALL_SLOTS
        buf = (ring[0] + k * _SMALL_SLOT, ring[1][k * _SMALL_SLOT:(k + 1) * _SMALL_SLOT])
        offs, off = [], 0
        for n in sizes:
            offs.append(off)
            off += (n + 15) & ~15
        srcs = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in self.ts])
        nb = (ctypes.c_uint64 * 8)(*sizes)
        of = (ctypes.c_uint64 * 8)(*offs)
        flag, k, seq = _hip.next_signal(d)
        _hip.call("mr_small_d2h", srcs, nb, of, len(self.ts), ctypes.c_void_p(buf[0]), flag, seq, _hip.stream(d))
        self.sig = (k, seq)
        self.views = [(buf[1], o, n, t) for o, n, t in zip(offs, sizes, self.ts)]

    def wait(self) -> list:
        if self.sig is None:
            return host_read_many(self.ts)
        _hip.spin(*self.sig, self.device)
        return [a[o:o + n].view(_NP_DTYPE[t.dtype]).reshape(tuple(t.shape)).copy() for a, o, n, t in self.views]


_SMALL_READ: dict = {}
_SMALL_SLOT, _SMALL_SLOTS = 1 << 14, 4  # bytes per read, reads outstanding at once


def host_read_begin(ts: list) -> HostRead:
    """Queue the download of small device tensors on the current stream;
    ``.wait()`` returns them as numpy arrays (one host wait)."""
    return HostRead(ts)


def host_read_many(ts: list) -> list:
    """Several small device tensors -> host numpy copies with ONE wait (the
    downloads are queued back to back on the current stream)."""
    if not ts or not ts[0].is_cuda:
        return [t.detach().numpy().copy() for t in ts]
    ts = [t.contiguous() for t in ts]
    sizes = [t.numel() * t.element_size() for t in ts]
    total = sum((n + 15) & ~15 for n in sizes)
    d = ts[0].device
    buf = _HOST_READ.get(d)
    if buf is None or buf.numel() < total:
        buf = torch.empty(max(total, 1 << 12), dtype=torch.uint8, pin_memory=True)
        _HOST_READ[d] = buf
    off = 0
    views = []
    for t, n in zip(ts, sizes):
        _hip.call("mr_d2h_async", _hip.ptr(buf[off:off + n]), _hip.ptr(t), n, _hip.stream(d))
        views.append((off, n, t))
        off += (n + 15) & ~15
    _hip.wait_stream(d)
    return [buf[o:o + n].numpy().view(_NP_DTYPE[t.dtype]).reshape(tuple(t.shape)).copy() for o, n, t in views]


_NP_DTYPE = {torch.int64: np.int64, torch.int32: np.int32, torch.uint8: np.uint8, torch.float32: np.float32,
             torch.float64: np.float64, torch.uint32: np.uint32, torch.int16: np.int16}


def copy_to_host(t: torch.Tensor, host: torch.Tensor, nelem: torch.Tensor) -> None:
    """Queue a device->pinned-host copy of ``nelem[0]`` elements of ``t``
    (count read on the device; no host synchronisation)."""
    _hip.call("mr_copy_to_host", _hip.ptr(t), _hip.ptr(host), _hip.ptr(nelem), t.element_size(),
              host.numel() * host.element_size(), _hip.stream(t.device))


_EPOCH = [0]
_SORT_WS: dict = {}


def _onesweep_tiles(n: int) -> int:
    """Tiles (= look-back granule rows) of one onesweep pass over n keys
    (csrc/hip/sort.hip mr_onesweep_tiles: 1024-key tiles up to 2^18 keys,
    4096 up to 2^22, 256 x MR_SORT_ROUNDS above)."""
    return int(_hip.lib().mr_onesweep_tiles(n))


def _sort_ws(d, n: int):
    """Per-device workspace for the onesweep sort (grown, never shrunk)."""
    tiles = _onesweep_tiles(n)
    ws = _SORT_WS.get(d)
    if ws is None or ws["tiles"] < tiles:
        ws = {"tiles": max(tiles, 64),
              "granules": torch.zeros(max(tiles, 64) * 256, dtype=torch.int64, device=d),
              "small": torch.zeros(2048 + 64 + 1, dtype=torch.int32, device=d)}
        _SORT_WS[d] = ws
    return ws


def sort_keys(words: list[torch.Tensor], bits: list[int] | None = None,
              return_keys: bool = False, ghist: torch.Tensor | None = None, from_bit: int = 0,
              keys_only: bool = False, runs: bool = False):
    """Stable permutation sorting rows by unsigned multi-word keys.

    ``words[0]`` is the most significant u64 word.  ``bits[j]`` limits the
    number of low bits of word j that participate (e.g. partition ids).
    Returns int32 (GPU) / int64 (CPU) permutation (and, with ``return_keys``,
    ``words[0]`` in sorted order as a second value).  ``ghist``: precomputed
    [8][256] digit histograms of a single-word key (skips that pass).  ``from_bit``
    (single word, GPU onesweep): only bits >= from_bit are sorted — rows equal
    in those bits keep their input order.  ``keys_only`` (single word, GPU
    onesweep): no permutation is carried (a third less traffic per pass);
    returns ``(None, sorted keys)``.  ``runs``: a hint that consecutive keys
    share digits (e.g. posting keys in text order) — the digit histograms then
    count each run once.  GPU: LSD radix sort, one onesweep launch per 8-bit
    digit (decoupled look-back, csrc/hip/sort.hip).
    """
    n = words[0].numel()
    bits = bits or [64] * len(words)
    if words[0].is_cuda:
        d = words[0].device
        if n == 0:
            z = torch.zeros(0, dtype=torch.int32, device=d)
            return (z, words[0][:0]) if return_keys else z
        lib = _hip.lib()
        s = _hip.stream(d)
        # onesweep LSD passes (csrc/hip/sort.hip)
        # no input copy and no iota launch: the first pass reads the
        # caller's word and generates the identity permutation itself
        ws = _sort_ws(d, n)
        small = ws["small"]
        small.zero_()  # [0:2048) ghist, [2048:2112) tile counters, [2112] error flag
        if torch.cuda.is_current_stream_capturing():
            # a replayed graph reuses its pass epochs: clear the look-back
            # granules so a replay never sees the previous replay's tags
            ws["granules"][: _onesweep_tiles(n) * 256].zero_()
        ghist_ws = small[:2048]
        pre_hist = ghist
        kbuf = [torch.empty(n, dtype=torch.int64, device=d) for _ in range(2)]
        pbuf = ([None, None] if keys_only and len(words) == 1
                else [torch.empty(n, dtype=torch.int32, device=d) for _ in range(2)])
        kin, pin = None, None
        pass_id = 0
        for j, (w, nb) in enumerate(zip(reversed(words), reversed(bits))):
            if pin is None:
                kin = w.contiguous()
            else:
                dst = kbuf[0] if kin is not kbuf[0] else kbuf[1]
                _hip.call("mr_gather_u64", _hip.ptr(w), _hip.ptr(pin), _hip.ptr(dst), n, s)
                kin = dst
            if nb <= 0:
                continue
            gh = ghist_ws
            if pre_hist is not None and len(words) == 1:
                gh = pre_hist
            else:
                if pass_id:
                    ghist_ws.zero_()
                d0 = from_bit // 8 if len(words) == 1 else 0  # digits below from_bit are not sorted
                _hip.call("mr_radix_ghist8", _hip.ptr(kin), n, _hip.ptr(ghist_ws),
                          (nb + 7) // 8 | (_GHIST_RUNS if runs else 0) | (d0 << 16), s)
            ko = keys_only and len(words) == 1
            for shift in range(from_bit if len(words) == 1 else 0, nb, 8):
                _EPOCH[0] = (_EPOCH[0] + 1) & 0xFFFFFF or 1
                kout = kbuf[0] if kin is not kbuf[0] else kbuf[1]
                pout = None if ko else (pbuf[0] if pin is not pbuf[0] else pbuf[1])
                _hip.call("mr_radix_onesweep_u32v", _hip.ptr(kin), _hip.ptr(pin), _hip.ptr(kout), _hip.ptr(pout),
                          n, shift, _hip.ptr(gh[shift // 8 * 256:]), _hip.ptr(ws["granules"]),
                          _hip.ptr(small[2048 + pass_id:]), _EPOCH[0], _hip.ptr(small[2112:]),
                          1 if (pin is None and not ko) else 0, s)
                pass_id += 1
                kin, pin = kout, pout
            if ko:
                return None, (kin if pass_id else words[0].clone())
        if pin is None:
            pin = torch.empty(n, dtype=torch.int32, device=d)
            _hip.call("mr_iota_u32", _hip.ptr(pin), n, s)
            kin = words[0].clone()
        return (pin, kin) if return_keys else pin
    cols = [_u64(w) for w in words]
    for j, nb in enumerate(bits):
        if nb < 64:
            cols[j] = cols[j] & np.uint64((1 << nb) - 1)
    perm = torch.from_numpy(np.lexsort(tuple(reversed(cols))).astype(np.int64))
    return (perm, words[0][perm]) if return_keys else perm


def sort_keys32(k32: torch.Tensor, ghist: torch.Tensor | None = None, bits: int = 32):
    """(permutation int32, sorted keys) of unsigned 32-bit keys (an int32
    tensor of bit patterns), stable.  GPU: one onesweep pass over u32 keys
    per 8-bit digit below ``bits`` (csrc/hip/sort.hip mr_radix_onesweep_k32);
    ``ghist``: the keys' digit histograms in the [8][256] layout (digit b at
    256 b), e.g. from records.keys32 — required on the GPU."""
    n = k32.numel()
    if not k32.is_cuda:
        u = k32.numpy().view(np.uint32).astype(np.uint64)
        if bits < 32:
            u &= np.uint64((1 << bits) - 1)
        perm = np.argsort(u, kind="stable").astype(np.int64)
        return torch.from_numpy(perm), k32[torch.from_numpy(perm)]
    d = k32.device
    if n == 0:
        return torch.zeros(0, dtype=torch.int32, device=d), k32[:0]
    if ghist is None:
        raise ValueError("sort_keys32 on the GPU needs the digit histograms (records.keys32 computes them)")
    s = _hip.stream(d)
    ws = _sort_ws(d, n)
    small = ws["small"]
    small[2048:].zero_()  # tile counters + error flag (the histograms are the caller's)
    kbuf = [torch.empty(n, dtype=torch.int32, device=d) for _ in range(2)]
    pbuf = [torch.empty(n, dtype=torch.int32, device=d) for _ in range(2)]
    kin, pin = k32.contiguous(), None
    for pass_id, shift in enumerate(range(0, bits, 8)):
        _EPOCH[0] = (_EPOCH[0] + 1) & 0xFFFFFF or 1
        kout = kbuf[0] if kin is not kbuf[0] else kbuf[1]
        pout = pbuf[0] if pin is not pbuf[0] else pbuf[1]
        _hip.call("mr_radix_onesweep_k32", _hip.ptr(kin), _hip.ptr(pin), _hip.ptr(kout), _hip.ptr(pout), n, shift,
                  _hip.ptr(ghist[shift // 8 * 256:]), _hip.ptr(ws["granules"]), _hip.ptr(small[2048 + pass_id:]),
                  _EPOCH[0], _hip.ptr(small[2112:]), 1 if pin is None else 0, s)
        kin, pin = kout, pout
    return pin, kin




def sort_by_partition_key(part: torch.Tensor, hi: torch.Tensor, lo: torch.Tensor, val: torch.Tensor,
                          rep: torch.Tensor, nparts: int, src: torch.Tensor | None = None):
    """Rows ordered by (partition, key) -> (part, hi, lo, val, rep, bad).

    GPU fast path (nparts <= 256): radix-sort ONE u64 composite word
    ``part << 56 | hi >> 8`` (8 passes instead of 17), reorder the columns with
    one gather launch, and insertion-sort the short runs that tie on it in a
    fixup kernel — by exact key order when the key bytes ``src`` are given
    (long keys sharing the 8-byte prefix compared bytewise on the device).
    ``bad`` (device int32): bit 0 = a run exceeded the fixup limit (caller must
    use the full multi-word sort); bit 1 = no ``src`` and a long-key prefix tie
    exists (the host must check those keys bytewise); bit 2 = the radix sort's
    look-back gave up (caller must re-sort).  CPU: lexsort (+bit 1).
    """
    n = hi.numel()
    if not hi.is_cuda or nparts > 256:
        perm = sort_keys([part.to(torch.int64), hi, lo], bits=[max(8, int(nparts - 1).bit_length()), 64, 64]).long()
        bad = torch.full((1,), 2, dtype=torch.int32, device=hi.device)
        return part[perm], hi[perm], lo[perm], val[perm], rep[perm], bad
    d = hi.device
    s = _hip.stream(d)
    part = part.to(torch.int32).contiguous()
    c = torch.empty(n, dtype=torch.int64, device=d)
    _hip.call("mr_composite_key", _hip.ptr(part), _hip.ptr(hi), n, _hip.ptr(c), s)
    perm, c = sort_keys([c], return_keys=True)
    cols = [torch.empty(n, dtype=torch.int64, device=d) for _ in range(4)]
    part2 = torch.empty(n, dtype=torch.int32, device=d)
    _hip.call("mr_gather_cols", _hip.ptr(perm), n, _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(val), _hip.ptr(rep), None,
              _hip.ptr(part), *[_hip.ptr(x) for x in cols], None, _hip.ptr(part2), s)
    hi, lo, val, rep = cols
    bad = torch.zeros(1, dtype=torch.int32, device=d)
    _hip.call("mr_tie_fixup", _hip.ptr(c), _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(val), _hip.ptr(rep), _hip.ptr(part2),
              n, _hip.ptr(bad), _hip.ptr(src) if src is not None else None, None, s)
    err = sort_error_word(d)
    if err is not None:  # bit 2: the sort's look-back gave up (order invalid)
        bad.bitwise_or_((err != 0).to(torch.int32) * 4)
    return part2, hi, lo, val, rep, bad


def sort_error(device) -> bool:
    """True if a onesweep look-back of the last sort_keys call on ``device``
    gave up (that sort's order is invalid).  Synchronises."""
    d = torch.device(device)
    ws = _SORT_WS.get(d)
    return bool(ws is not None and int(ws["small"][2112].item()) != 0)


def sort_error_word(device) -> torch.Tensor | None:
    """Device int32[1] error word of the last sort_keys call (no sync)."""
    d = torch.device(device)
    ws = _SORT_WS.get(d)
    return None if ws is None else ws["small"][2112:2113]


EXACT_MAX_WORDS = 32  # keys up to 256 bytes get the device's exact order


def key_word(hi: torch.Tensor, lo: torch.Tensor, rep: torch.Tensor, src: torch.Tensor | None,
             k: int) -> torch.Tensor:
    """Bytes [8k, 8k+8) of every key as a big-endian int64 word, zero padded
    past the key's end (so unsigned word order is byte order).  ``hi`` None:
    word 0 of long keys read from their bytes too (spans with no key words,
    e.g. byte-string values)."""
    n = lo.numel()
    if hi is None and not lo.is_cuda:
        hi = torch.zeros_like(lo)
    if lo.is_cuda:
        d = lo.device
        w = torch.empty(n, dtype=torch.int64, device=d)
        if n:
            _hip.call("mr_key_word", _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep), _hip.ptr(src), n, k, _hip.ptr(w),
                      _hip.stream(d))
        return w
    out = np.zeros(n, np.uint64)
    for i, b in enumerate(key_bytes_list(hi, lo, rep, src)):
        out[i] = int.from_bytes(b[8 * k:8 * k + 8].ljust(8, b"\0"), "big")
    return torch.from_numpy(out.view(np.int64))


def _alpha_words(k7, alpha: list, nparts: int):
    """The exact sort's words re-coded to the byte values present
    (csrc/hip/keyops.hip pack_alpha_kernel) when that takes fewer radix passes
    than the 7-bit words' 15: ([word0, word1], bits, partition bits), or
    (None, None, 8).  Codes keep the byte order (zero padding -> 0), so the
    sorted order is the same."""
    present = [b for b in range(1, 128) if alpha[b >> 5] >> (b & 31) & 1]
    cbits = max(1, len(present).bit_length())
    pb = int(max(nparts, 1) - 1).bit_length()
    if cbits >= 7 or pb > 8:
        return None, None, 8
    c0 = min((64 - pb) // cbits, 16)
    rest = (16 - c0) * cbits
    passes = 8 + (rest + 7) // 8
    if passes >= 15 or rest > 64:
        return None, None, 8
    code = np.zeros(128, np.uint8)
    code[present] = np.arange(1, len(present) + 1, dtype=np.uint8)
    d = k7[0].device
    out = torch.empty((2, k7[0].shape[1]), dtype=torch.int64, device=d)
    _hip.call("mr_pack_alpha", _hip.ptr(k7[0]), k7[0].shape[1], _hip.ptr(torch.from_numpy(code).to(d)), cbits, pb,
              _hip.ptr(out), _hip.stream(d))
    words, bits = ([out[0], out[1]], [64, rest]) if rest else ([out[0]], [64])
    return words, bits, pb


def exact_key_perm(part: torch.Tensor, hi: torch.Tensor, lo: torch.Tensor, rep: torch.Tensor,
                   src: torch.Tensor | None, nparts: int, klen: torch.Tensor | None = None,
                   with_part: bool = False, with_counts: bool = False, w1: torch.Tensor | None = None,
                   k7=None, perm32: bool = False):
    """Stable permutation ordering rows by (partition, exact key bytes) on the
    device, for key sets the (partition, hi, lo) sort plus the tie fix-up
    cannot order (long keys — whose lo is a hash — in long runs of a shared
    8-byte prefix, e.g. n-grams).

    MSD refinement over 16-byte windows of the key (mr_key_word; zero padded):
    round 0 sorts every row by (partition, bytes 0-15, min(len, 16)); a key of
    at most 16 bytes is then placed exactly (a shorter key that is a prefix of a
    longer one sorts first through the length column).  Only rows that still
    tie — long keys sharing their first 16 bytes — go to the next round, which
    sorts them by (tie group, bytes 16-31, min(len, 32)) in place inside their
    groups, and so on.  Each round is a stable LSD radix sort, so rows of one
    key set keep their input order where they tie.  None when a key is longer
    than 8 * EXACT_MAX_WORDS bytes (the caller orders on the host).
    ``klen``: the keys' lengths when the caller has them (key_meta); ``w1``:
    their ``key_word(..., 1)`` likewise (key_meta(want_w1=True)); ``perm32``
    (GPU): the permutation as the sort's int32 (no int64 round trip for a
    caller whose gathers take int32 rows); ``k7``:
    key_meta(want_k7=True)'s 7-bit sort words and flag — when every key's
    first 16 bytes are 7-bit, the GPU sort of keys past 16 bytes runs over
    those two words (15 passes and one gather instead of 17 and two: the
    partition rides in the top byte).
    ``with_part``: return (perm, partitions in the new order as int64) —
    the sort's major word, so no gather is needed for it.  ``with_counts``
    (GPU): also the rows per partition (int64 [nparts]), which the sort's
    digit histogram of its partition word already holds.

    Keys longer than 16 bytes go through the tie fix-up below, which orders
    rows equal in (partition, bytes 0-15) by their full bytes and then their
    lengths; for them the GPU sort leaves the length column out (one pass,
    its histograms and a gather fewer) and falls back to the four-column
    sort only when a tie run is too long for the fix-up."""
    n = hi.numel()
    d = hi.device
    if n == 0:
        z = torch.zeros(0, dtype=torch.int64, device=d)
        return (z, z.clone()) if with_part else z
    if klen is None:
        _, klen = key_meta(hi, lo, rep, src, want_part=False)
    klen = klen.to(torch.int64)
    alpha = None
    if k7 is not None:  # the longest key, the 7-bit flag and the byte alphabet in one read
        extra = [k7[2].to(torch.int64)] if len(k7) > 2 and k7[2] is not None else []
        got = host_read(torch.cat([torch.stack([klen.max(), k7[1][0].to(torch.int64)])] + extra))
        max_len, k7_bad = int(got[0]), int(got[1])
        if extra:
            alpha = [int(x) & 0xFFFFFFFF for x in got[2:6]]
    else:
        max_len, k7_bad = int(klen.max()), 1
    if (max_len + 7) // 8 > EXACT_MAX_WORDS:
        return None
    pbits = max(8, int(max(nparts, 1) - 1).bit_length())
    if w1 is None:
        w1 = key_word(hi, lo, rep, src, 1)
    cols_ = []

    def cols():
        # (partition, hi, w1, min(len, 16)): built when a path sorts by them
        # (the 7-bit / alphabet words need none of the four conversions)
        if not cols_:
            cols_.extend([part.to(torch.int64), hi, w1, klen.clamp(max=16)])
        return cols_
    counts = None

    def sort_cols(cs, bits):
        nonlocal counts
        out = sort_keys_checked(cs, bits=bits, return_keys=True)
        if with_counts and hi.is_cuda and pbits == 8:  # the partition word's digit histogram (sort_keys' workspace)
            counts = _SORT_WS[d]["small"][:max(nparts, 1)].to(torch.int64)
        return out

    def done(p):
        # every later step reorders rows only inside runs of one partition
        if perm32 and p.is_cuda:
            p = p if p.dtype == torch.int32 else p.to(torch.int32)
        elif p.dtype != torch.int64:
            p = p.long()
        out = (p, spart) if with_part else p
        if with_counts:
            c = counts if counts is not None else bincount(spart, max(nparts, 1))
            out = (*out, c) if with_part else (out, c)
        return out

    if max_len <= 16 or not hi.is_cuda:
        p32, spart = sort_cols(cols(), [pbits, 64, 64, 8])
        if max_len <= 16:
            return done(p32)
    elif not k7_bad and pbits == 8:
        words, bits, pb = _alpha_words(k7, alpha, nparts) if alpha is not None else (None, None, 8)
        if words is None:
            # 7-bit keys: (partition, bytes 0-15) as two words of 64 and 56 bits
            words, bits = [k7[0][0], k7[0][1]], [64, 56]
        p32, sk = sort_keys_checked(words, bits=bits, return_keys=True)
        spart = ((sk >> (64 - pb)) & ((1 << pb) - 1)) if pb else torch.zeros_like(sk)
        if with_counts:  # the top digit's histogram of the last word sorted: partitions in its top pb bits
            top = _SORT_WS[d]["small"][7 * 256:8 * 256].to(torch.int64)
            counts = top.view(1 << pb, 1 << (8 - pb)).sum(1)[:max(nparts, 1)] if pb else top.sum().view(1)
    else:
        p32, spart = sort_cols(cols()[:3], [pbits, 64, 64])
    if hi.is_cuda:
        # runs of rows equal in the sort columns (long keys sharing 16 bytes),
        # found through a hash of the columns in sorted order and insertion-
        # sorted by their full bytes and lengths, one thread per run
        # (mr_exact_fix); runs longer than its limit go to the refinement
        # rounds below, after the four-column sort
        s = _hip.stream(d)
        part32 = part.to(torch.int32).contiguous()
        h = torch.empty(n, dtype=torch.int64, device=d)
        _hip.call("mr_exact_hash", _hip.ptr(part32), _hip.ptr(hi), _hip.ptr(w1), None, n, _hip.ptr(h), s)
        sh = torch.empty(n, dtype=torch.int64, device=d)
        _hip.call("mr_gather_u64", _hip.ptr(h), _hip.ptr(p32), _hip.ptr(sh), n, s)
        bad = torch.zeros(1, dtype=torch.int32, device=d)
        _hip.call("mr_exact_fix", _hip.ptr(sh), _hip.ptr(p32), n, _hip.ptr(part32), _hip.ptr(hi), _hip.ptr(w1),
                  _hip.ptr(klen), _hip.ptr(rep), _hip.ptr(src), _hip.ptr(bad), s)
        if not int(bad.item()):
            return done(p32)
        p32, spart = sort_cols(cols(), [pbits, 64, 64, 8])
    perm = p32.long()
    scols = [c[perm] for c in cols()]
    pos = torch.arange(n, dtype=torch.int64, device=d)
    cap = 16
    while True:
        # ties: adjacent rows equal in every column whose keys go on past cap
        same = scols[-1][1:] == cap
        for c in scols:
            same &= c[1:] == c[:-1]
        if not bool(same.any()):
            return done(perm)
        member = torch.zeros(pos.numel(), dtype=torch.bool, device=d)
        member[1:] |= same
        member[:-1] |= same
        head = torch.ones(pos.numel(), dtype=torch.int64, device=d)
        head[1:] = (~same).to(torch.int64)
        grp = torch.cumsum(head, 0)[member]
        grp = grp - grp[:1]
        pos = pos[member]
        rows = perm[pos]
        k = cap // 8
        rh, rl, rr = hi[rows], lo[rows], rep[rows]
        cap += 16
        rcols = [grp, key_word(rh, rl, rr, src, k), key_word(rh, rl, rr, src, k + 1), klen[rows].clamp(max=cap)]
        gbits = max(8, int(grp[-1]).bit_length())
        sub = sort_keys_checked(rcols, bits=[gbits, 64, 64, max(8, cap.bit_length())]).long()
        perm[pos] = rows[sub]  # a group's rows stay inside its positions (grp is the major column)
        scols = [c[sub] for c in rcols]


def sort_keys_checked(words, bits=None, retries: int = 2, **kw):
    """sort_keys that checks the look-back error word (one host sync) and
    re-sorts on a give-up; raises after ``retries`` failed re-sorts."""
    for attempt in range(retries + 1):
        out = sort_keys(words, bits, **kw)
        if not words[0].is_cuda or not sort_error(words[0].device):
            return out
    raise RuntimeError("radix sort: decoupled look-back gave up %d times" % (retries + 1))


def debug_sort_fail(passes: int) -> None:
    """Test knob: the next ``passes`` onesweep passes give up one look-back."""
    _hip.call("mr_sort_debug_fail", int(passes))


def bincount(ids: torch.Tensor, nbins: int) -> torch.Tensor:
    if ids.is_cuda:
        if DEBUG_CHECKS and ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= nbins):
            raise RuntimeError(f"bincount: ids out of [0, {nbins})")
        d = ids.device
        out = torch.zeros(nbins, dtype=torch.int64, device=d)
        _hip.call("mr_bincount", _hip.ptr(ids), ids.numel(), nbins, _hip.ptr(out), _hip.stream(d))
        return out
    return torch.bincount(ids.long(), minlength=nbins)[:nbins]


def reduce_by_key(hi: torch.Tensor, lo: torch.Tensor | None, vals: torch.Tensor | None, op: str = "sum",
                  rep: torch.Tensor | None = None):
    """Fold runs of equal (hi, lo) in SORTED input -> (uhi, ulo, uval, urep, start)."""
    n = hi.numel()
    if hi.is_cuda:
        d = hi.device
        s = _hip.stream(d)
        heads = torch.empty(n, dtype=torch.int32, device=d)
        _hip.call("mr_segment_heads", _hip.ptr(hi), _hip.ptr(lo), n, _hip.ptr(heads), s)
        seg, total = exclusive_scan(heads)
        m = int(total.item()) if n else 0
        uhi = torch.empty(m, dtype=torch.int64, device=d)
        ulo = torch.empty(m, dtype=torch.int64, device=d) if lo is not None else None
        urep = torch.empty(m, dtype=torch.int64, device=d) if rep is not None else None
        start = torch.empty(m, dtype=torch.int64, device=d)
        uval = torch.full((m,), _op_init(op), dtype=torch.int64, device=d)
        _hip.call("mr_segment_keys", _hip.ptr(seg), _hip.ptr(heads), _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep), n,
                  _hip.ptr(uhi), _hip.ptr(ulo), _hip.ptr(urep), _hip.ptr(start), s)
        _hip.call("mr_segment_fold", _hip.ptr(seg), _hip.ptr(heads), _hip.ptr(vals), n, OPS[op], _hip.ptr(uval), s)
        return uhi, ulo, uval, urep, start
    h = _u64(hi)
    lw = _u64(lo) if lo is not None else np.zeros_like(h)
    if n == 0:
        z = torch.zeros(0, dtype=torch.int64)
        return z, (z.clone() if lo is not None else None), z.clone(), (z.clone() if rep is not None else None), z
    heads = np.ones(n, bool)
    heads[1:] = (h[1:] != h[:-1]) | (lw[1:] != lw[:-1])
    start = np.flatnonzero(heads)
    v = _np(vals).astype(np.int64) if vals is not None else np.ones(n, np.int64)
    ufunc = {"sum": np.add, "min": np.minimum, "max": np.maximum}[op]
    uval = ufunc.reduceat(v, start)
    return (_t64(h[start]), _t64(lw[start]) if lo is not None else None, torch.from_numpy(uval),
            _t64(_u64(rep)[start]) if rep is not None else None, torch.from_numpy(start.astype(np.int64)))
