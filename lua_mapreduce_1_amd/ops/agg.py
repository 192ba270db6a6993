"""Key -> typed value columns / value lists on the device (HIP kernels in
``csrc/hip/generic.hip``; NumPy on CPU tensors — the executable
specification).  The storage of the general device plane
(parallel/generic.py).

The reference groups every emitted value under its key and lets the reducer
(or the combiner of the reduce module) fold the list
(/root/reference/mapreduce/job.lua:83-112, task.lua:325).  Here a key maps to a
slot of an HBM hash table (the 128-bit keys of ops/keys.py, long keys
verified byte for byte) and each slot holds either

* K typed value columns folded in place (``fold`` mode): the column spec
  ``"<dtype>:<op>"`` with dtype ``i64`` (default) / ``f64`` / ``f32`` and op
  ``sum | min | max | count | mean`` (``mean`` is kept as a sum and a count
  and divided when results are read), or
* the list of every value emitted for it (``list`` mode): postings
  (slot, value) appended in emission order.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _hip
from . import keys as K
from .primitives import HashTable, _np, _t64, _u64, next_pow2

DTYPES = {"i64": torch.int64, "f64": torch.float64, "f32": torch.float32}
_VT = {torch.int64: 0, torch.float64: 1, torch.float32: 2, torch.int32: 3}
_VT_SCALAR = 4
_OPC = {"sum": 0, "min": 1, "max": 2}
OPS = ("sum", "min", "max", "count", "mean")
MAXC = 8
_I64_MAX, _I64_MIN = (1 << 63) - 1, -(1 << 63)


class ColSpec:
    """One output column of a fold: dtype + op (``count`` is int64)."""

    __slots__ = ("dtype", "op")

    def __init__(self, dtype: str, op: str):
        if op not in OPS:
            raise ValueError(f"unknown fold op {op!r} (one of {OPS})")
        if dtype not in DTYPES:
            raise ValueError(f"unknown column dtype {dtype!r} (one of {tuple(DTYPES)})")
        if op == "count":
            dtype = "i64"
        if op == "mean":
            dtype = "f64"
        self.dtype, self.op = dtype, op

    def __repr__(self):
        return f"{self.dtype}:{self.op}"

    def __eq__(self, o):
        return isinstance(o, ColSpec) and (self.dtype, self.op) == (o.dtype, o.op)


def parse_spec(spec) -> list[ColSpec]:
    """``"f64:sum"``, ``"max"``, ``("f64:mean", "f64:max", "count")``, ... ->
    column specs (dtype defaults to i64)."""
    items = [spec] if isinstance(spec, str) else list(spec)
    out = []
    for it in items:
        if isinstance(it, ColSpec):
            out.append(it)
            continue
        parts = str(it).split(":")
        if len(parts) == 1:
            out.append(ColSpec("i64", parts[0]))
        elif len(parts) == 2:
            a, b = parts
            out.append(ColSpec(a, b) if a in DTYPES else ColSpec(b, a))
        else:
            raise ValueError(f"bad column spec {it!r}")
    if not out or len(out) > MAXC:
        raise ValueError(f"a fold has 1..{MAXC} columns (got {len(out)})")
    return out


def is_column_spec(spec) -> bool:
    """True for specs the general plane folds (typed or several columns);
    plain ``"sum" | "min" | "max" | "count"`` stay on the int64 fold plane."""
    if spec is None:
        return False
    if isinstance(spec, str):
        if spec in ("sum", "min", "max", "count"):
            return False
        try:
            parse_spec(spec)
            return True
        except ValueError:
            return False
    try:
        parse_spec(spec)
        return True
    except (ValueError, TypeError):
        return False


class Physical:
    """Physical columns of a list of output specs: (dtype, fold op, input
    index or None for the constant 1).  ``mean`` = f64 sum + i64 count."""

    def __init__(self, specs: list[ColSpec]):
        self.specs = specs
        self.cols: list[tuple[str, str, int | None]] = []
        self.out: list[tuple] = []  # per output: ("col", j) | ("mean", j_sum, j_cnt)

        def col(c) -> int:
            # one physical column per distinct (dtype, op, input): a mean and
            # a count share their count (one atomic fewer per row)
            if c not in self.cols:
                self.cols.append(c)
            return self.cols.index(c)
        for i, s in enumerate(specs):
            if s.op == "mean":
                self.out.append(("mean", col(("f64", "sum", i)), col(("i64", "sum", None))))
            elif s.op == "count":
                self.out.append(("col", col(("i64", "sum", None))))
            else:
                self.out.append(("col", col((s.dtype, s.op, i))))
        if len(self.cols) > MAXC:
            raise ValueError(f"at most {MAXC} physical columns (means count twice)")

    @property
    def n_in(self) -> int:
        return len(self.specs)

    def outputs(self, cols: list) -> list:
        """Output columns (numpy or torch) from physical ones."""
        res = []
        for o in self.out:
            if o[0] == "col":
                res.append(cols[o[1]])
            else:
                s, c = cols[o[1]], cols[o[2]]
                if isinstance(s, torch.Tensor):
                    res.append(s / c.to(torch.float64))
                else:
                    with np.errstate(invalid="ignore", divide="ignore"):
                        res.append(s / c.astype(np.float64))
        return res


def _identity(dtype: str, op: str):
    if op == "sum":
        return 0
    if dtype == "i64":
        return _I64_MAX if op == "min" else _I64_MIN
    return float("inf") if op == "min" else float("-inf")


class _ColsArg(ctypes.Structure):
    _fields_ = [("k", ctypes.c_longlong), ("list", ctypes.c_longlong), ("src", ctypes.c_void_p * MAXC),
                ("stype", ctypes.c_longlong * MAXC), ("sbits", ctypes.c_longlong * MAXC),
                ("dst", ctypes.c_void_p * MAXC), ("dtype", ctypes.c_longlong * MAXC),
                ("op", ctypes.c_longlong * MAXC), ("post_slot", ctypes.c_void_p), ("post_base", ctypes.c_ulonglong),
                ("rows_only", ctypes.c_longlong), ("cstride", ctypes.c_longlong)]


class _CsvArg(ctypes.Structure):
    _fields_ = [("sep", ctypes.c_longlong), ("kf", ctypes.c_longlong), ("nin", ctypes.c_longlong),
                ("vf", ctypes.c_longlong * MAXC), ("pin", ctypes.c_longlong * MAXC)]


CSV_MAXV = 4  # value inputs of the fused CSV fold (csrc/hip/generic.hip CV_MAXV)


def _scalar_bits(v, dtype: str) -> int:
    if dtype == "i64":
        return int(v)
    if dtype == "f64":
        return int(np.array([float(v)], np.float64).view(np.int64)[0])
    return int(np.array([float(v)], np.float32).view(np.int32)[0])


class AggTable:
    """Keys -> slots of an HBM table plus per-slot value columns (fold) or
    an append-only posting sink (list).  ``cols`` = physical columns
    ``[(dtype, op, input index | None)]`` (fold mode) or None (list mode,
    values of ``list_dtype``).  ``src``: the byte source every rep word
    indexes (set by the owner before inserting long keys)."""

    def __init__(self, capacity: int, device, cols: list | None = None, list_dtype="i64", runs: bool = False):
        from ..parallel.values import spec_of
        self.device = torch.device(device)
        self.cols_spec = cols
        self.list_mode = cols is None
        # list mode: a posting's value row (parallel/values.py: numbers,
        # tuples, byte-string span words); list_dtype the legacy scalar name
        self.vspec = spec_of(list_dtype)
        self.list_dtype = self.vspec.dtype
        self.src: torch.Tensor | None = None
        self.cap = next_pow2(max(1024, int(capacity)))
        self.cstride = 1  # slot stride of the value columns (one array per column)
        if self.is_cuda:
            self.keys = HashTable(self.cap, self.device, op="none")
            self.cols = [] if self.list_mode else [torch.empty(self.cap, dtype=DTYPES[dt], device=self.device)
                                                   for dt, _op, _i in cols]
            self._fill_cols()
            self.post_slot = self.post_val = None
        else:
            self._pending: list = []
        self.npost = 0
        # Run-length postings (list mode on the GPU, one scalar value column):
        # while every row inserted so far carries the SAME constant value (a
        # word count's emit(word, 1)), a key's list is that constant repeated,
        # so the table keeps a per-slot COUNT (an LDS-combined fold) instead
        # of one (slot, value) posting per row — no posting writes, no posting
        # sort and gather before the combiner.  The first row with another
        # value expands the counts into postings (every earlier row precedes
        # it, so each list's emission order is kept) and the table continues
        # as plain list mode.  Opt-in (``runs``): expanded postings keep each
        # list's order but not the rows' global order, which a caller pairing
        # postings with its input rows (the shuffle's receive table) needs.
        from ..utils.config import TUNABLES
        self._runs_opt = bool(runs)
        self._runs = self._runs_opt and self.is_cuda and self.list_mode and self.vspec.scalar and TUNABLES.const_runs
        self.run_bits: int | None = None  # the constant's value bits (None: no row yet)
        self._run_count: torch.Tensor | None = None

    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def _fill_cols(self) -> None:
        for c, (dt, op, _i) in zip(self.cols, self.cols_spec or []):
            c.fill_(_identity(dt, op))

    def reset(self) -> None:
        self.src = None
        self.npost = 0
        if self.is_cuda:
            self.keys.reset()
            self._fill_cols()
            from ..utils.config import TUNABLES
            self._runs = self._runs_opt and self.list_mode and self.vspec.scalar and TUNABLES.const_runs
            if self.run_bits is not None and self._run_count is not None:
                self._run_count.zero_()
            self.run_bits = None
        else:
            self._pending = []

    # -- run-length postings ---------------------------------------------------
    @property
    def runs(self) -> bool:
        """True while the postings are held as per-slot counts of one constant."""
        return self._runs and self.run_bits is not None

    def _run_insert(self, vals: list) -> bool:
        """Whether this insert's rows can be counted (run-length form): one
        scalar value equal to every earlier row's.  Leaves the run form
        (expanding it) when not."""
        if not self._runs:
            return False
        v, dt = vals[0]
        if len(vals) == 1 and not isinstance(v, torch.Tensor):
            bits = _scalar_bits(v, dt)
            if self.run_bits is None or self.run_bits == bits:
                if self._run_count is None:
                    self._run_count = torch.zeros(self.cap, dtype=torch.int64, device=self.device)
                self.run_bits = bits
                return True
        self.expand_runs()
        return False

    def expand_runs(self) -> None:
        """Counts -> explicit postings (slot, constant); plain list mode from here."""
        if not self._runs:
            return
        self._runs = False
        if self.run_bits is None:
            return  # nothing counted yet
        slot, _hi, _lo, _rep, _ = self.compact()
        cnt = self._run_count[slot]
        n = int(cnt.sum())
        self.npost = 0
        self._grow_posts(n)
        if n:
            self.post_slot[:n] = torch.repeat_interleave(slot, cnt, output_size=n)
            self.post_val[:n].fill_(self.run_bits)
        self.npost = n

    def run_count(self, slot: torch.Tensor) -> torch.Tensor:
        """Run-length form: the rows counted for each key slot."""
        return self._run_count[slot]

    def run_lists(self, known: tuple[int, bool] | None = None):
        """Run-length form: (slot, hi, lo, rep) of every key and its list in
        CSR form (off [m + 1], val: the constant repeated) — what
        parallel/reducers.lists_of_postings builds from explicit postings,
        without the sort."""
        slot, hi, lo, rep, _ = self.compact(known)
        cnt = self._run_count[slot]
        off = torch.zeros(slot.numel() + 1, dtype=torch.int64, device=self.device)
        torch.cumsum(cnt, 0, out=off[1:])
        n = int(off[-1]) if slot.numel() else 0
        return slot, hi, lo, rep, off, torch.full((n,), self.run_bits, dtype=torch.int64, device=self.device)  # value bits

    # -- inserts ---------------------------------------------------------------
    def _values(self, values, n: int) -> list:
        """Per physical column (src tensor | None, scalar bits)."""
        if self.list_mode:
            sp = self.vspec
            if len(values) > sp.width:
                raise ValueError(f"{len(values)} value columns emitted, the value lists hold {sp}")
            out = []
            for j, dt in enumerate(sp.cols):
                if j >= len(values) and dt == "bytes":
                    raise ValueError(f"value column {j} ({sp}) is a byte string: emit it (ByteSpans)")
                # byte columns arrive as int64 span words (GenericEmitter)
                out.append((values[j] if j < len(values) else 1, "i64" if dt == "bytes" else dt))
            return out
        out = []
        for dt, _op, i in self.cols_spec:
            v = 1 if i is None else values[i]
            out.append((v, dt))
        return out

    def _grow_posts(self, need: int) -> None:
        if self.post_slot is None or self.post_slot.numel() < need:
            k = self.vspec.width
            cap = max(need, 2 * (self.post_slot.numel() if self.post_slot is not None else 0), 1 << 16)
            ns = torch.empty(cap, dtype=torch.int64, device=self.device)
            nv = torch.empty(cap * k, dtype=torch.int64, device=self.device)  # value rows [cap][k]
            if self.post_slot is not None and self.npost:
                ns[:self.npost].copy_(self.post_slot[:self.npost])
                nv[:self.npost * k].copy_(self.post_val[:self.npost * k])
            self.post_slot, self.post_val = ns, nv

    def insert(self, n: int, values, hi=None, lo=None, rep=None, rep_add: int = 0, text=None, starts=None,
               lens=None, rep_base: int = 0) -> None:
        """Insert n rows: keys pre-encoded (hi, lo, rep + rep_add) or byte
        spans (starts, lens) of ``text`` (rep offset = rep_base + start);
        ``values``: one tensor (length n) or scalar per input column."""
        if n == 0:
            return
        vals = self._values(values, n)
        if self.is_cuda and self.list_mode and self._run_insert(vals):
            a = _ColsArg()  # the rows' key counts: a fold (LDS-combined) into the run-count column
            a.k, a.list, a.cstride, a.rows_only = 1, 0, 1, 0
            a.stype[0], a.sbits[0], a.dtype[0], a.op[0] = _VT_SCALAR, 1, _VT[torch.int64], _OPC["sum"]
            a.dst[0] = self._run_count.data_ptr()
            self._agg_insert(a, n, [], hi, lo, rep, rep_add, text, starts, lens, rep_base)
            self.npost += n
            return
        if self.is_cuda:
            a = _ColsArg()
            a.k = len(vals)
            a.list = 1 if self.list_mode else 0
            a.cstride = 1 if self.list_mode else self.cstride
            # (list mode: one row per thread; an LDS key -> slot cache and batched
            # rows per thread measured slower, profiles/r4/pruned/; a direct
            # per-row insert without the LDS combine and a sort-based
            # pre-combine lost too, profiles/r5/pruned/)
            a.rows_only = 0
            keep = []
            for j, (v, dt) in enumerate(vals):
                if isinstance(v, torch.Tensor):
                    if v.numel() != n:
                        raise ValueError(f"value column {j}: {v.numel()} values for {n} keys")
                    if v.device != self.device:
                        v = v.to(self.device)
                    if v.dtype not in _VT:
                        v = v.to(torch.float64 if v.is_floating_point() else torch.int64)
                    v = v.contiguous()
                    keep.append(v)
                    a.src[j] = v.data_ptr()
                    a.stype[j] = _VT[v.dtype]
                else:
                    a.stype[j] = _VT_SCALAR
                    a.sbits[j] = _scalar_bits(v, dt)
                a.dtype[j] = _VT[DTYPES[dt]]
                a.op[j] = _OPC[self.cols_spec[j][1]] if not self.list_mode else 0
                if not self.list_mode:
                    a.dst[j] = self.cols[j].data_ptr()
            if self.list_mode:
                self._grow_posts(self.npost + n)
                a.dst[0] = self.post_val.data_ptr()
                a.post_slot = self.post_slot.data_ptr()
                a.post_base = self.npost
            self._agg_insert(a, n, keep, hi, lo, rep, rep_add, text, starts, lens, rep_base)
            self.npost += n if self.list_mode else 0
            return
        # CPU: pending rows, folded at compaction
        if text is not None:
            buf = _np(text)
            st = _np(starts).astype(np.int64)
            ln = _np(lens).astype(np.int64)
            ok = (ln > 0) & (st >= 0)
            h, lw = K.span_keys(buf, np.where(ok, st, 0), np.where(ok, ln, 1))
            r = ((st.astype(np.uint64) + np.uint64(rep_base)) << np.uint64(K.REP_LEN_BITS)) | \
                np.minimum(np.maximum(ln, 0), K.REP_LEN_MASK).astype(np.uint64)
        else:
            h, lw = _u64(hi).copy(), _u64(lo).copy()
            r = _u64(rep).copy() if rep is not None else np.zeros(n, np.uint64)
            if rep is not None and rep_add:
                r = r + np.uint64(rep_add << K.REP_LEN_BITS)
            ok = np.ones(n, bool)
        cols = []
        for v, dt in vals:
            npdt = {"i64": np.int64, "f64": np.float64, "f32": np.float32}[dt]
            cols.append(_np(v).astype(npdt) if isinstance(v, torch.Tensor) else np.full(n, v, npdt))
        self._pending.append((h, lw, r, cols, ok, ok))
        self.npost += n if self.list_mode else 0

    def _agg_insert(self, a, n: int, keep: list, hi, lo, rep, rep_add, text, starts, lens, rep_base) -> None:
        t = self.keys
        if text is not None:
            st = starts.to(torch.int64).contiguous()
            ln = lens.to(torch.int32).contiguous()
            keep += [st, ln]
            _hip.call("mr_agg_insert", *t._gtab(), t.cap, _hip.ptr(self.src), None, None, None, 0,
                      _hip.ptr(text), _hip.ptr(st), _hip.ptr(ln), rep_base, n, ctypes.byref(a),
                      _hip.stream(self.device))
        else:
            _hip.call("mr_agg_insert", *t._gtab(), t.cap, _hip.ptr(self.src), _hip.ptr(hi.contiguous()),
                      _hip.ptr(lo.contiguous()), _hip.ptr(rep.contiguous()) if rep is not None else None,
                      rep_add, None, None, None, 0, n, ctypes.byref(a), _hip.stream(self.device))

    def insert_keys(self, hi, lo, rep) -> None:
        """List mode: keys with NO posting (a key whose combiner emitted
        nothing keeps its place, like the reference's ``return k,{}`` line of
        an emptied list, job.lua:198-214): the key is in the table, its list
        is empty."""
        n = int(hi.numel())
        if n == 0:
            return
        if self.is_cuda:
            self.keys.insert(hi.contiguous(), lo.contiguous(), torch.zeros(n, dtype=torch.int64, device=self.device),
                             rep.contiguous(), src=self.src)
            return
        k = self.vspec.width
        self._pending.append((_u64(hi).copy(), _u64(lo).copy(), _u64(rep).copy(), [np.zeros(n, np.int64)] * k,
                              np.ones(n, bool), np.zeros(n, bool)))

    def insert_csv(self, text: torch.Tensor, rep_base: int, key: int, values, sep: int,
                   rows_out: torch.Tensor) -> None:
        """Fold mode on the GPU: every line of ``text`` -> key = field ``key``,
        input i = the number in field ``values[i]`` (None: the constant 1),
        folded by the fused kernel (mr_csv_fold: lines, fields, parse and the
        LDS-combined insert in one pass over the bytes); rows with a missing
        or empty key or a value that does not parse are dropped.
        ``rows_out`` (int64 [1], device) += the rows folded."""
        if not self.is_cuda or self.list_mode:
            raise ValueError("insert_csv: a fold-mode table on the GPU")
        if len(values) > CSV_MAXV or max([key] + [v for v in values if v is not None]) >= 1 << 20:
            raise ValueError(f"insert_csv: at most {CSV_MAXV} value fields")
        sa = _CsvArg()
        sa.sep, sa.kf, sa.nin = int(sep) & 0xFF, int(key), len(values)
        for i, v in enumerate(values):
            sa.vf[i] = -1 if v is None else int(v)
        keep: list = []
        vals = []
        for j, (dt, _op, i) in enumerate(self.cols_spec):
            sa.pin[j] = -1 if i is None else int(i)
            vals.append((1 if i is None else 0.0, dt))  # field inputs: no source array (the kernel parses)
        a = self._cols_arg(vals, 0, keep)
        t = self.keys
        _hip.call("mr_csv_fold", *t._gtab(), t.cap, _hip.ptr(self.src), _hip.ptr(text), text.numel(), rep_base,
                  ctypes.byref(sa), ctypes.byref(a), _hip.ptr(rows_out), _hip.stream(self.device))

    def _cols_arg(self, vals: list, n: int, keep: list):
        a = _ColsArg()
        a.k = len(vals)
        a.list = 0
        a.cstride = self.cstride
        for j, (v, dt) in enumerate(vals):
            if isinstance(v, torch.Tensor):
                if v.numel() != n:
                    raise ValueError(f"value column {j}: {v.numel()} values for {n} keys")
                if v.dtype not in _VT:
                    v = v.to(torch.float64 if v.is_floating_point() else torch.int64)
                v = v.contiguous()
                keep.append(v)
                a.src[j] = v.data_ptr()
                a.stype[j] = _VT[v.dtype]
            else:
                a.stype[j] = _VT_SCALAR
                a.sbits[j] = _scalar_bits(v, dt)
            a.dtype[j] = _VT[DTYPES[dt]]
            a.op[j] = _OPC[self.cols_spec[j][1]]
            a.dst[j] = self.cols[j].data_ptr()
        return a

    def rehome_long_keys(self, buf: torch.Tensor, lo_off: int, hi_off: int, heap: torch.Tensor,
                         heap_cap: int) -> None:
        """Streaming map rounds: the bytes of the long keys whose rep points
        into buf[lo_off:hi_off) move to the key heap at the front of ``buf``
        (``heap`` = int64[2] bump counter + full flag) and their reps follow
        (HashTable.rehome_long_keys for the GPU key table)."""
        if self.is_cuda:
            self.keys.rehome_long_keys(buf, lo_off, hi_off, heap, heap_cap)
            return
        b = _np(buf)
        h = heap.numpy()
        for hi_, lo_, r, _cols, ok, _post in self._pending:
            long_ = ok & ((lo_ & np.uint64(0xFF)) == np.uint64(K.LONG_MARK))
            off = r >> np.uint64(K.REP_LEN_BITS)
            for i in np.flatnonzero(long_ & (off >= np.uint64(lo_off)) & (off < np.uint64(hi_off))):
                o, n = int(r[i]) >> K.REP_LEN_BITS, int(r[i]) & K.REP_LEN_MASK
                d = int(h[0])
                if d + n > heap_cap:
                    h[1] = 1
                    continue
                b[d:d + n] = b[o:o + n].copy()
                h[0] = d + n
                r[i] = np.uint64(K.make_rep(d, n))

    # -- state -----------------------------------------------------------------
    def stats(self) -> tuple[int, bool]:
        if self.is_cuda:
            return self.keys.stats()
        return sum(int(p[4].sum()) for p in self._pending), False

    def _cpu_ids(self):
        """CPU: (unique keys (hi, lo, rep), inverse ids of the valid pending rows, valid rows' cols)."""
        if not self._pending:
            z = np.zeros(0, np.uint64)
            return z, z, z, np.zeros(0, np.int64), None
        ok = np.concatenate([p[4] for p in self._pending])
        hi = np.concatenate([p[0] for p in self._pending])[ok]
        lo = np.concatenate([p[1] for p in self._pending])[ok]
        r = np.concatenate([p[2] for p in self._pending])[ok]
        cols = [np.concatenate([p[3][j] for p in self._pending])[ok] for j in range(len(self._pending[0][3]))]
        keys = np.empty(hi.size, dtype=[("hi", np.uint64), ("lo", np.uint64), ("d", np.int64)])
        keys["hi"], keys["lo"], keys["d"] = hi, lo, 0
        long_ = (lo & np.uint64(0xFF)) == np.uint64(K.LONG_MARK)
        if long_.any() and self.src is not None:
            sb = _np(self.src)
            ids: dict = {}
            dcol = keys["d"]
            for i in np.flatnonzero(long_):
                rr = int(r[i])
                o, ln = rr >> K.REP_LEN_BITS, rr & K.REP_LEN_MASK
                dcol[i] = ids.setdefault(sb[o:o + ln].tobytes(), len(ids) + 1)
        uk, first, inv = np.unique(keys, return_index=True, return_inverse=True)
        return uk["hi"].copy(), uk["lo"].copy(), r[first], inv.astype(np.int64), cols

    def compact(self, known: tuple[int, bool] | None = None):
        """Fold mode: (slot, hi, lo, rep, [physical cols]) of every key, dense
        (arbitrary order on the GPU, key order on the CPU)."""
        if self.is_cuda:
            n, ovf = known if known is not None else self.stats()
            if ovf:
                raise OverflowError("aggregation table overflow")
            t = self.keys
            d = self.device
            slot, hi, lo, rep = (torch.empty(n, dtype=torch.int64, device=d) for _ in range(4))
            counter = torch.zeros(1, dtype=torch.int64, device=d)
            _hip.call("mr_slot_compact", *t._gtab(), t.cap, _hip.ptr(slot), _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep),
                      _hip.ptr(counter), _hip.stream(d))
            cols = [c[slot] for c in self.cols]
            return slot, hi, lo, rep, cols
        h, lw, r, inv, cols = self._cpu_ids()
        m = h.size
        out = []
        if not self.list_mode and cols is not None:
            for (dt, op, _i), v in zip(self.cols_spec, cols):
                npdt = v.dtype
                agg = np.full(m, _identity(dt, op), npdt)
                {"sum": np.add, "min": np.minimum, "max": np.maximum}[op].at(agg, inv, v)
                out.append(torch.from_numpy(agg))
        elif not self.list_mode:
            out = [torch.from_numpy(np.full(0, _identity(dt, op), {"i64": np.int64, "f64": np.float64,
                                                                     "f32": np.float32}[dt]))
                   for dt, op, _i in self.cols_spec]
        slot = torch.arange(m, dtype=torch.int64)
        return slot, _t64(h), _t64(lw), _t64(r), out

    def postings(self):
        """List mode: (slot, hi, lo, rep) of every key and the (posting slot,
        posting value) pairs in emission order (slot -1: dropped row) — for a
        table that counted runs, each key's postings in order, keys grouped."""
        if self.is_cuda:
            self.expand_runs()
            slot, hi, lo, rep, _ = self.compact()
            n = self.npost
            sp = self.vspec
            if n == 0:
                z = torch.zeros(0, dtype=torch.int64, device=self.device)
                return slot, hi, lo, rep, z, sp.storage(z.clone())
            return slot, hi, lo, rep, self.post_slot[:n], sp.storage(self.post_val[:n * sp.width])
        h, lw, r, inv, cols = self._cpu_ids()
        if any(not p[5].all() for p in self._pending):
            # key-only rows (insert_keys): in the key set, no posting
            post = np.concatenate([p[5] for p in self._pending])[np.concatenate([p[4] for p in self._pending])]
            inv = np.where(post, inv, -1)
        sp = self.vspec
        bits = [c.view(np.int64) if c.dtype == np.float64 else c.astype(np.int64, copy=False) for c in cols or []]
        if not bits:
            bits = [np.zeros(0, np.int64)] * sp.width
        vals = bits[0] if sp.scalar else np.stack(bits, 1)
        return (torch.arange(h.size, dtype=torch.int64), _t64(h), _t64(lw), _t64(r), torch.from_numpy(inv),
                torch.from_numpy(np.ascontiguousarray(vals)))
