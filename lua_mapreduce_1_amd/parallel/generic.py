"""General device MapReduce plane: any keys, typed folds, value lists, or the
user's own reducefn — so a job that is not word count, word -> lines or
TeraSort still runs its map, grouping and shuffle on the GPU.

The reference's contract (/root/reference/mapreduce/job.lua:83-112,264-284):
``mapfn`` emits (key, value) pairs, values are grouped per key, the combiner
(taken from the reduce module, task.lua:325) and the reducer fold each key's
list.  Here a ``device_mapfn(key, data, emit)`` picks keys and values out of
the staged bytes with torch ops and ops/text.py, and emits them in batches:

* ``emit.spans(starts, lens, *values, text=None)`` — key i = the bytes
  ``text[starts[i] : starts[i] + lens[i]]`` (default ``text``: the staged
  chunk being mapped); empty spans (len <= 0) are skipped;
* ``emit.pairs(hi, lo, *values, rep=None, src=None)`` — keys already encoded
  (ops/keys.py), long keys' bytes located by ``rep`` in ``src``;
* ``emit.words(text=None, *values)`` — every whitespace token (value 1 by
  default); ``emit.word_lines(text=None)`` — every token with the global
  number of its line (the inverted index's pairs);
* ``emit(key, *values)`` — one host pair (buffered, inserted in one batch).

``values``: one tensor (one value per key) or Python number per input column.
What happens to them is the reduce module's ``device_reduce``:

* a column spec, ``"f64:sum"``, ``("f64:mean", "f64:max", "count")``, ...
  (ops/agg.py) — each key's values are folded in place into typed columns
  (native f64/f32/i64 atomics); the result of a key is the list of its
  output columns, like a reducefn that emits several values;
* ``"concat"`` / ``"concat_unique"`` — the key's values in emission order /
  sorted and distinct (int64, float64, a k-tuple of numbers or a byte string,
  as the map module's ``device_value_dtype`` declares: parallel/values.py);
* absent — the values are grouped on the device (list, emission order) and
  the module's own ``reducefn(key, values, emit)`` runs on the host for each
  key of the rank's partitions (the reduce job), skipping singleton lists
  when the reducer declares all three ACI flags (job.lua:264-274).  Nothing
  is folded with an op the user did not declare.

Map-side grouping happens in ONE HBM table per rank (the combiner of
job.lua:92-96 becomes the fold); the shuffle sends each key (with its folded
columns or its value list) to the rank owning its partition ``p % W`` in one
count exchange and three ``all_to_all_single``; the reduce side merges what
it receives in a second table and orders the keys by (partition, key bytes).
"""
from __future__ import annotations

import contextlib
import sys
import time
import traceback

import numpy as np
import torch

from .. import ops, utils
from ..ops import agg as A
from ..ops import keys as K
from ..ops import primitives as P
from ..ops import segments as S
from ..ops import text as TX
from ..runtime import codec
from ..runtime import device as devmod
from ..runtime import modules
from ..utils import STATUS
from ..utils import trace
from ..utils.config import TUNABLES
from . import dist as D
from . import reducers as RD
from . import values as VL

_BIG_TABLE = 1 << 24  # (slots) map tables this large are refitted from 2x their fit, not 4x


def _bits(n: int) -> int:
    return max(1, int(max(n, 1) - 1).bit_length())


class NeedsHostMap(Exception):
    """A device map called an emitter that this execution mode cannot run
    (the caller runs the host ``mapfn`` instead)."""


class StreamedSourceError(ValueError):
    """A streamed map (arena_cap_mb) emitted keys that are not spans of its
    staged input (raised to the caller, not treated as a failing job)."""


# ---------------------------------------------------------------------------
class KeySource:
    """The ONE byte source every rep word of an iteration's table indexes:
    the engine's staged input arena (keys are spans of the input, read in
    place), extended on demand by a copy of the arena followed by appended
    bytes (host keys, spans of derived tensors)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.begin(None)

    fixed = False  # a streamed map: the source is the engine's ring buffer, nothing may be appended

    def begin(self, arena) -> None:
        self.arena = arena
        self.buf = None
        self.used = arena.numel() if arena is not None else 0

    def set_arena(self, arena) -> None:
        if self.arena is None and self.buf is None and arena is not None:
            self.begin(arena)

    def _base(self):
        return self.buf if self.buf is not None else self.arena

    def offset_of(self, t: torch.Tensor) -> int | None:
        """Byte offset of ``t`` inside the source (None: not a view of it).
        Once bytes were appended the source is a copy ``buf`` whose first
        ``arena.numel()`` bytes mirror the arena at the same offsets, so a
        view of the arena keeps its arena offset."""
        if t.dtype != torch.uint8:
            return None
        for b, lim in ((self.buf, self.used), (self.arena, self.arena.numel() if self.arena is not None else 0)):
            if b is None or t.device != b.device:
                continue
            p = t.data_ptr() - b.data_ptr()
            if 0 <= p and p + t.numel() <= lim:
                if b is self.arena and self.buf is not None and t.numel():
                    # staged after the copy was taken: refresh its mirror
                    self.buf[p:p + t.numel()].copy_(t.reshape(-1), non_blocking=True)
                return p
        return None

    def add(self, t: torch.Tensor) -> tuple[int, torch.Tensor]:
        """Append ``t``'s bytes; returns (offset, the source's view of them)."""
        t = t.reshape(-1)
        if t.dtype != torch.uint8:
            raise TypeError("key bytes must be a uint8 tensor")
        if self.fixed:
            raise StreamedSourceError("a streamed general-plane map (arena_cap_mb) emits spans of its staged input "
                                      "only (no host keys or spans of other tensors)")
        n = t.numel()
        need = self.used + n
        if self.buf is None or self.buf.numel() < need:
            cap = max(need, 2 * (self.buf.numel() if self.buf is not None else 0), self.used + (1 << 16))
            nb = torch.empty(cap, dtype=torch.uint8, device=self.device)
            if self.buf is not None:
                nb[:self.used].copy_(self.buf[:self.used])
            elif self.arena is not None and self.used:
                nb[:self.used].copy_(self.arena[:self.used])
            self.buf = nb
        off = self.used
        if n:
            self.buf[off:need].copy_(t, non_blocking=True)
        self.used = need
        return off, self.buf[off:need]

    def locate(self, t: torch.Tensor) -> tuple[torch.Tensor, int]:
        """(device view of t's bytes inside the source, its offset)."""
        off = self.offset_of(t)
        if off is not None:
            return t, off
        off, view = self.add(t)
        return view, off

    def source(self) -> torch.Tensor:
        b = self._base()
        if b is None:
            return torch.zeros(1, dtype=torch.uint8, device=self.device)
        return b[:max(self.used, 1)] if self.used else b[:1]


class GenericEmitter:
    """``emit`` of a general device map (see the module docstring)."""

    def __init__(self, mapper: "GenericMap"):
        self.m = mapper
        self.chunk: torch.Tensor | None = None
        self.line_base = None  # callable: global line number of the chunk's first byte
        self.err_word = None

    @property
    def device(self):
        return self.m.device

    def _text(self, text):
        t = self.chunk if text is None else text
        if t is None:
            raise ValueError("no staged chunk: pass text=")
        if t.device != self.m.device:
            t = t.to(self.m.device)
        return t

    def spans(self, starts, lens, *values, text=None) -> None:
        t, base = self.m.src.locate(self._text(text))
        self.m.insert(int(starts.numel()), values, text=t, starts=starts, lens=lens, rep_base=base)

    def bytes(self, starts, lens, text=None) -> VL.ByteSpans:
        """A byte-string value column for ``spans`` / ``pairs``: value i =
        ``text[starts[i] : starts[i] + lens[i]]`` (default ``text``: the
        chunk being mapped); needs ``device_value_dtype`` "bytes" there."""
        return VL.ByteSpans(starts, lens, self._text(text) if text is not None else None)

    def pairs(self, hi, lo, *values, rep=None, src=None) -> None:
        add = 0
        if src is not None:
            _, add = self.m.src.locate(src if src.device == self.m.device else src.to(self.m.device))
        elif rep is not None and self.chunk is not None:
            add = self.m.src.offset_of(self.chunk)  # rep words relative to the mapped chunk
            if add is None:
                raise ValueError("emit.pairs(rep=...): the mapped chunk is not part of the key source; pass src= "
                                 "(the tensor the rep words index)")
        self.m.insert(int(hi.numel()), values, hi=hi, lo=lo, rep=rep, rep_add=add)

    def csv(self, text=None, key: int = 0, values=(1,), sep=",") -> None:
        """Every line of the chunk (or ``text``) as one row: key = field
        ``key`` (``sep``-separated, 0-based), value input i = the number in
        field ``values[i]`` (None: the constant 1); rows whose key is missing
        or empty or whose value fields do not parse are dropped.  Typed folds
        on the GPU run one fused kernel (lines, fields, parse and the
        LDS-combined insert); otherwise the ops/text.py chain."""
        t = self._text(text)
        self.m.insert_csv(t, int(key), tuple(values), sep if isinstance(sep, int) else ord(sep))

    def words(self, text=None, *values) -> None:
        t = self._text(text)
        st, ln = TX.tokens(t)
        self.spans(st, ln, *values, text=t)

    def word_lines(self, text=None) -> None:
        """Every whitespace token of the chunk with the global (0-based)
        number of the line it is on (needs split inputs: line numbers are
        global over every split)."""
        if self.line_base is None:
            raise NeedsHostMap("word_lines needs the SPMD engine's global line numbering")
        t = self._text(text)
        st, ln, line = TX.tokens(t, lines=True)
        line = line + self.line_base(t)  # an int, or a device scalar
        self.spans(st, ln, line, text=t)

    def records(self, *a, **k):
        raise NeedsHostMap("emit.records needs the record plane (device_reduce = 'identity')")

    def error_word(self):
        return self.err_word

    def __call__(self, key, *values) -> None:
        if isinstance(key, str):
            key = key.encode("utf-8", "surrogateescape")
        elif not isinstance(key, bytes):
            key = str(key).encode()
        if not key:
            return
        self.m.host.append((key, values))


class GenericMap:
    """Map-side state of the general plane: the key -> columns / postings
    table, the byte source of its rep words and the emitter."""

    def __init__(self, device, capacity: int, phys: A.Physical | None, list_dtype="i64",
                 reducers: "RD.ListReducers | None" = None, combine_at: int = 0):
        self.device = torch.device(device)
        self.phys = phys
        self.vspec = VL.spec_of(list_dtype)  # list mode: the value row of a posting
        self.list_dtype = self.vspec.dtype
        self.table = self.new_table(capacity)
        self.src = KeySource(self.device)
        self.emit = GenericEmitter(self)
        self.host: list = []
        self._rows_dev = None
        self.rows = 0
        # list mode with a combiner: the table's postings are combined
        # whenever they pass combine_at (the batched MAX_MAP_RESULT,
        # job.lua:92-96) and once more at the end of the map (job.lua:198-202)
        self.reducers = reducers if (reducers is not None and reducers.has_combiner and phys is None) else None
        self.combine_at = int(combine_at or TUNABLES.combine_postings)
        # the next combine runs when the postings pass this: after a combine
        # (or a refused one) it moves to twice what is left, so a combiner
        # that cannot shrink the table (many distinct keys, a dedup or top-k
        # combiner) runs O(log n) times per map, not once per emit call
        self._next_combine = self.combine_at
        self.combines = 0

    def new_table(self, capacity: int) -> A.AggTable:
        """The map's key table: typed fold columns, or value lists (run-length
        postings while the values are one constant, ops/agg.py)."""
        return A.AggTable(capacity, self.device, self.phys.cols if self.phys is not None else None, self.vspec,
                          runs=True)

    @property
    def n_in(self) -> int:
        return self.phys.n_in if self.phys is not None else self.vspec.width

    def _byte_words(self, v):
        """An emitted ByteSpans value column -> span words into the key
        source (the value text located there like key text)."""
        if not isinstance(v, VL.ByteSpans):
            return v
        if self.phys is not None:
            raise TypeError("byte-string values go to value lists (no device_reduce, or concat): a typed fold "
                            "folds numbers")
        text = v.text if v.text is not None else self.emit._text(None)
        _, base = self.src.locate(text)
        return VL.span_words(v.starts.to(self.device), v.lens.to(self.device), base)

    def add_bytes(self, data) -> int:
        """Append bytes (a uint8 tensor or bytes) to the key source; returns
        their offset (byte-string values made by a combiner or host emits)."""
        if not isinstance(data, torch.Tensor):
            data = torch.frombuffer(bytearray(data), dtype=torch.uint8) if len(data) else \
                torch.zeros(0, dtype=torch.uint8)
        off, _ = self.src.add(data.to(self.device))
        return off

    def begin(self, arena=None) -> None:
        self.table.reset()
        self.src.begin(arena)
        self.host = []
        self.rows = 0
        self.combines = 0

    def insert(self, n: int, values, **kw) -> None:
        if n == 0:
            return
        if len(values) > self.n_in or (self.phys is not None and len(values) not in (0, self.n_in)):
            raise ValueError(f"{len(values)} value columns emitted, the reduce expects {self.n_in}")
        if self.phys is not None and not values:
            values = (1,) * self.n_in
        if self.vspec.has_bytes:
            values = tuple(self._byte_words(v) for v in values)
        self.table.src = self.src.source()
        self.table.insert(n, list(values), **kw)
        self.rows += n
        if self.reducers is not None and self.table.npost >= self._next_combine:
            self.combine()
            self._next_combine = max(self.combine_at, 2 * self.table.npost)

    def insert_csv(self, text: torch.Tensor, key: int, values: tuple, sep: int) -> None:
        fused = (self.phys is not None and self.table.is_cuda and len(values) <= A.CSV_MAXV
                 and len(values) == self.n_in)
        if not fused:
            ks, kl, cols = TX.csv_rows(text, key, values, sep)
            t, base = self.src.locate(text)
            self.insert(int(ks.numel()), tuple(cols), text=t, starts=ks, lens=kl, rep_base=base)
            return
        t, base = self.src.locate(text)
        if self._rows_dev is None:
            self._rows_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.table.src = self.src.source()
        self.table.insert_csv(t, base, key, values, sep, self._rows_dev)

    @property
    def rows(self) -> int:
        """Rows emitted into the table (the fused CSV fold counts its rows on
        the device: read here, once per iteration)."""
        if self._rows_dev is not None:
            self._rows += int(self._rows_dev.item())
            self._rows_dev = None
        return self._rows

    @rows.setter
    def rows(self, v: int) -> None:
        self._rows = int(v)
        self._rows_dev = None

    def combine(self) -> bool:
        """Run the reduce module's combiner over every key's list and rebuild
        the table from the combined postings (same capacity, same key
        source).  False (nothing done) when the table overflowed: the map is
        re-run with a larger one anyway."""
        t = self.table
        if self.reducers is None or t.npost == 0:
            return False
        m, ovf = t.stats()
        if ovf or (t.is_cuda and m > t.cap // 2 + 1):  # (CPU stats count rows: no capacity to respect)
            return False
        src = self.src.source()
        if t.runs and self.reducers.combiner_fold is not None:
            return self._combine_runs(t, (m, ovf))
        if t.runs:  # run-length postings: the lists straight from the per-key counts
            slot, hi, lo, rep, off, val = t.run_lists((m, ovf))
        else:
            slot, hi, lo, rep, pslot, pval = t.postings()
            m = int(hi.numel())
            space = t.cap if t.is_cuda else max(1, m)
            off, val = RD.lists_of_postings(slot, pslot, pval, m, space)
        noff, nval = self.reducers.combine(RD.KeyBatch(hi, lo, rep, src), off, val, src=src,
                                           add_bytes=self.add_bytes)
        nt = self.new_table(t.cap)
        nt.src = self.src.source()  # (a combiner may have appended byte values)
        n = int(noff[-1]) if noff.numel() else 0
        if n:
            kid = S.ids(noff, n)
            nt.insert(n, self._value_cols(nval), hi=hi[kid], lo=lo[kid], rep=rep[kid])
        empty = S.lengths(noff) == 0
        if bool(empty.any()):
            # a key whose combiner emitted nothing stays, with an empty list:
            # the reference still writes it (`return k,{}`, job.lua:198-214),
            # so its reducer runs over whatever the other maps sent
            nt.insert_keys(hi[empty], lo[empty], rep[empty])
        self.table = nt
        self.combines += 1
        return True

    def _combine_runs(self, t, known) -> bool:
        """A recognised fold combiner over run-length postings: key i's list
        is the constant c repeated cnt[i] times, so its combined value is
        c * cnt[i] (sum, int64) or c (min / max) — singleton lists unchanged,
        keys with an empty list kept empty — without materialising the lists."""
        slot, hi, lo, rep, _ = t.compact(known)
        cnt = t.run_count(slot)
        has = cnt > 0
        c = torch.tensor(t.run_bits, dtype=torch.int64, device=self.device)
        nval = (c * cnt[has]) if self.reducers.combiner_fold == "sum" else c.expand(int(has.sum())).clone()
        nt = self.new_table(t.cap)
        nt.src = self.src.source()
        n = int(nval.numel())
        if n:
            nt.insert(n, self._value_cols(nval), hi=hi[has], lo=lo[has], rep=rep[has])
        if not bool(has.all()):
            e = ~has
            nt.insert_keys(hi[e], lo[e], rep[e])
        self.table = nt
        self.combines += 1
        return True

    def _value_cols(self, bits: torch.Tensor) -> list:
        """Stored value bits [n] / [n, k] -> the insert's value columns
        (float64 tensors for f64 columns: the kernel converts by type)."""
        rows = self.vspec.rows(bits)
        return [rows[:, j].contiguous().view(torch.float64) if dt == "f64" else rows[:, j].contiguous()
                for j, dt in enumerate(self.vspec.cols)]

    def flush_host(self) -> None:
        if not self.host:
            return
        pairs, self.host = self.host, []
        blob = b"".join(k for k, _ in pairs)
        base, _ = self.src.add(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.device))
        his, los, reps, off = [], [], [], 0
        for k, _ in pairs:
            h, l_ = K.pack_key(k)
            his.append(h)
            los.append(l_)
            reps.append(K.make_rep(base + off, len(k)))
            off += len(k)
        t64 = lambda a: torch.from_numpy(np.array(a, dtype=np.uint64).view(np.int64)).to(self.device)  # noqa: E731
        if self.phys is None and not self.vspec.scalar:
            # tuples / byte strings: one value row per pair (strings appended
            # to the key source as span words)
            vals = [v if len(v) != 1 else v[0] for _, v in pairs]
            bits = VL.host_bits(vals, self.vspec, self.add_bytes, "emit")
            cols = self._value_cols(torch.from_numpy(bits).to(self.device))
            self.insert(len(pairs), tuple(cols), hi=t64(his), lo=t64(los), rep=t64(reps))
            return
        k_in = max(len(v) for _, v in pairs) if self.phys is None else self.n_in
        cols = []
        for j in range(k_in):
            col = [v[j] if j < len(v) else 1 for _, v in pairs]
            isf = any(isinstance(x, float) for x in col)
            cols.append(torch.tensor(col, dtype=torch.float64 if isf else torch.int64, device=self.device))
        self.insert(len(pairs), tuple(cols), hi=t64(his), lo=t64(los), rep=t64(reps))


# ---------------------------------------------------------------------------
def _value_order_key(v: torch.Tensor, dtype: str) -> torch.Tensor:
    """int64 whose unsigned order is the numeric order of the values (value
    bit patterns: int64, or float64 when ``dtype`` is f64)."""
    sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=v.device)
    if dtype == "f64":
        neg = v < 0
        return torch.where(neg, ~v, v ^ sign)
    return v ^ sign


def order_fold(slot, hi, lo, rep, cols, src, nparts: int, partmod, phys: A.Physical, outputs: bool = True) -> dict:
    """Keys of a folded table in (partition, key) order with their output
    columns (``outputs=False``: the physical ones, e.g. a mean's sum and
    count for a later merge), on the device: {hi, lo, key_off, key_blob,
    cols, counts}."""
    m = hi.numel()
    d = hi.device
    part = devmod.partition_of(hi, lo, rep, src, nparts, partmod) if m else torch.zeros(0, dtype=torch.int32, device=d)
    exact = True
    if m:
        perm, exact = _key_order(part, hi, lo, rep, src, nparts)
        hi, lo, rep, part = hi[perm], lo[perm], rep[perm], part[perm]
        cols = [c[perm] for c in cols]
    _, klen = ops.key_meta(hi, lo, rep, src, want_part=False)
    koff, kblob = ops.gather_key_bytes(hi, lo, rep, src, lengths=klen)
    counts = ops.bincount(part, nparts) if m else torch.zeros(nparts, dtype=torch.int64, device=d)
    return {"hi": hi, "lo": lo, "key_off": koff, "key_blob": kblob, "cols": phys.outputs(cols) if outputs else cols,
            "counts": counts, "exact": exact}


def _key_order(part, hi, lo, rep, src, nparts: int):
    """(permutation into (partition, exact key bytes) order, True) on the
    device (ops.exact_key_perm: long keys sharing a prefix are placed by
    their bytes, not their hash) — or, for a key past the exact sort's length
    limit, the (partition, hi, lo) order and False (host_partitions then
    fixes the order of long keys sharing an 8-byte prefix)."""
    perm = ops.exact_key_perm(part, hi, lo, rep, src, nparts) if src is not None else None
    if perm is not None:
        return perm.long(), True
    return ops.sort_keys_checked([part.to(torch.int64), hi, lo], bits=[max(8, _bits(nparts)), 64, 64]).long(), False


def order_lists(slot, hi, lo, rep, pslot, pval, src, nparts: int, partmod, unique: bool, dtype,
                slot_space: int, vsrc=None) -> dict:
    """Keys in (partition, key) order with their value lists (emission order,
    or sorted distinct with ``unique``): {hi, lo, key_off, key_blob,
    list_off, list_val, counts} — or, for tuple / byte-string values
    (parallel/values.py), ``list_cols`` (one typed tensor per number column,
    a ByteValues per byte column, in posting order) instead of ``list_val``.
    ``vsrc``: the byte source of byte-string values (default ``src``)."""
    spec = VL.spec_of(dtype)
    vsrc = src if vsrc is None else vsrc
    m = hi.numel()
    d = hi.device
    part = devmod.partition_of(hi, lo, rep, src, nparts, partmod) if m else torch.zeros(0, dtype=torch.int32, device=d)
    exact = True
    if m:
        perm, exact = _key_order(part, hi, lo, rep, src, nparts)
        hi, lo, rep, part, slot = hi[perm], lo[perm], rep[perm], part[perm], slot[perm]
    rank = torch.full((max(slot_space, 1),), -1, dtype=torch.int64, device=d)
    rank[slot] = torch.arange(m, dtype=torch.int64, device=d)
    keep = pslot >= 0
    pr = rank[pslot.clamp(min=0)]
    keep &= pr >= 0
    pr, pv = pr[keep], pval[keep]
    if pr.numel():
        if unique:
            pr, pv = _unique_values(pr, pv, spec, m, vsrc)
        else:
            pp = ops.sort_keys_checked([pr], bits=[_bits(m)]).long()  # stable: emission order per key
            pr, pv = pr[pp], pv[pp]
    nper = torch.bincount(pr, minlength=m)[:m] if m else torch.zeros(0, dtype=torch.int64, device=d)
    loff = torch.zeros(m + 1, dtype=torch.int64, device=d)
    if m:
        loff[1:] = torch.cumsum(nper, 0)
    _, klen = ops.key_meta(hi, lo, rep, src, want_part=False)
    koff, kblob = ops.gather_key_bytes(hi, lo, rep, src, lengths=klen)
    counts = ops.bincount(part, nparts) if m else torch.zeros(nparts, dtype=torch.int64, device=d)
    out = {"hi": hi, "lo": lo, "key_off": koff, "key_blob": kblob, "list_off": loff, "counts": counts,
           "exact": exact}
    if spec.scalar:
        out["list_val"] = pv
    else:
        out["list_cols"] = list(_user_cols(pv, spec, vsrc))
    return out


def _user_cols(bits, spec: VL.ValueSpec, vsrc):
    """Stored value rows -> per column: a typed tensor, or ByteValues."""
    rows = spec.rows(bits)
    for j, dt in enumerate(spec.cols):
        col = rows[:, j].contiguous()
        yield VL.byte_values(col, vsrc) if dt == "bytes" else (col.view(torch.float64) if dt == "f64" else col)


def _unique_values(pr, pv, spec: VL.ValueSpec, m: int, vsrc):
    """Postings sorted by (key, value) with duplicates of a key's value
    dropped: numbers (scalars or tuples) in numeric order, one byte-string
    column in exact byte order (ops.exact_key_perm over the value bytes)."""
    d = pr.device
    if spec.scalar:
        pp = ops.sort_keys_checked([pr, _value_order_key(pv, spec.cols[0])], bits=[_bits(m), 64]).long()
        pr, pv = pr[pp], pv[pp]
        first = torch.ones(pr.numel(), dtype=torch.bool, device=d)
        first[1:] = (pr[1:] != pr[:-1]) | (pv[1:] != pv[:-1])
        return pr[first], pv[first]
    rows = spec.rows(pv)
    if spec.has_bytes:
        if spec.width != 1:
            raise ValueError("concat_unique: byte-string values are compared alone (device_value_dtype 'bytes'), "
                             "not inside tuples")
        w = rows[:, 0].contiguous()
        n = w.numel()
        z = torch.zeros(n, dtype=torch.int64, device=d)
        mark = torch.full((n,), 0xFF, dtype=torch.int64, device=d)
        vh = P.key_word(None, mark, w, vsrc, 0)  # the value's first 8 bytes (the key encoding's hi)
        pp = ops.exact_key_perm(pr, vh, mark, w, vsrc, max(m, 1))
        if pp is None:
            raise ValueError("concat_unique: a byte-string value is longer than the exact sort handles")
        pr, w, vh = pr[pp], w[pp], vh[pp]
        ln = VL.word_lengths(w)
        same = (pr[1:] == pr[:-1]) & (ln[1:] == ln[:-1]) & (vh[1:] == vh[:-1])
        for k in range(1, (int(ln.max()) + 7) // 8 if n else 0):
            wk = P.key_word(z, mark, w, vsrc, k)
            same &= wk[1:] == wk[:-1]
        first = torch.ones(n, dtype=torch.bool, device=d)
        first[1:] = ~same
        return pr[first], spec.storage(w[first].reshape(-1, 1))
    words = VL.order_words(rows, spec)
    pp = ops.sort_keys_checked([pr] + words, bits=[_bits(m)] + [64] * len(words)).long()
    pr, rows = pr[pp], rows[pp]
    first = torch.ones(pr.numel(), dtype=torch.bool, device=d)
    first[1:] = (pr[1:] != pr[:-1]) | (rows[1:] != rows[:-1]).any(1)
    return pr[first], spec.storage(rows[first])


def _np64(t):
    return t.detach().cpu().numpy()


def _np_cols(out: dict) -> list:
    return [_np64(c) for c in out.get("cols", [])]


def _host_list_cols(out: dict) -> list:
    """``list_cols`` on the host: numpy arrays, (off, blob) per byte column."""
    cols = []
    for c in out["list_cols"]:
        if isinstance(c, (VL.ByteValues, tuple)) and not isinstance(c, torch.Tensor):
            cols.append((_np64(c[0]).astype(np.int64), _np64(c[1])))
        else:
            cols.append(_np64(c))
    return cols


def _take_cols(cols: list, idx: np.ndarray) -> list:
    """Postings ``idx`` of host list columns (byte columns re-packed)."""
    out = []
    for c in cols:
        if isinstance(c, tuple):
            off, blob = c
            lens = off[idx + 1] - off[idx]
            noff = np.zeros(idx.size + 1, np.int64)
            np.cumsum(lens, out=noff[1:])
            if idx.size and np.all(np.diff(idx) == 1):
                nb = blob[off[idx[0]]:off[idx[-1] + 1]]
            else:
                b = blob.tobytes()
                nb = np.frombuffer(b"".join(b[off[i]:off[i + 1]] for i in idx), np.uint8)
            out.append((noff, nb))
        else:
            out.append(c[idx])
    return out


def host_values(cols: list) -> list:
    """Host list columns -> one Python value per posting: a number or a str
    (one column), or a tuple of them."""
    py = []
    for c in cols:
        if isinstance(c, tuple):
            off, blob = c
            b = blob.tobytes()
            py.append([codec.key_str(b[off[i]:off[i + 1]]) for i in range(off.size - 1)])
        else:
            py.append(c.tolist())
    return py[0] if len(py) == 1 else list(zip(*py))


def host_partitions(out: dict, nparts: int, dtype="i64", reducefn=None, aci: bool = False) -> dict:
    """Device result of :func:`order_fold` / :func:`order_lists` -> per
    partition host columns (exact bytewise key order inside a partition),
    with ``reducefn`` applied per key to list results (the host reduce)."""
    hi = _np64(out["hi"]).view(np.uint64)
    lo = _np64(out["lo"]).view(np.uint64)
    koff = _np64(out["key_off"]).astype(np.int64)
    kblob = _np64(out["key_blob"])
    counts = _np64(out["counts"])
    bounds = np.zeros(nparts + 1, np.int64)
    np.cumsum(counts, out=bounds[1:])
    cols = [_np64(c) for c in out.get("cols", [])]
    is_list = "list_off" in out
    lcols = None
    if is_list:
        loff = _np64(out["list_off"]).astype(np.int64)
        if "list_cols" in out:  # tuple / byte-string values (parallel/values.py)
            lcols = _host_list_cols(out)
        else:
            lval = _np64(out["list_val"])
            if VL.spec_of(dtype).dtype == "f64" and not out.get("list_typed"):
                lval = lval.view(np.float64)
    parts = {}
    kb = kblob.tobytes()
    exact = bool(out.get("exact", False))
    for p in range(nparts):
        a, b = int(bounds[p]), int(bounds[p + 1])
        if b <= a:
            continue
        fix = devmod.fix_long_key_order(hi[a:b], lo[a:b], koff[a:b + 1], kblob) if b - a > 1 and not exact else None
        idx = np.arange(a, b) if fix is None else fix + a
        if fix is None:
            k_off = koff[a:b + 1] - koff[a]
            k_blob = kblob[koff[a]:koff[b]]
        else:
            lens = (koff[idx + 1] - koff[idx])
            k_off = np.zeros(idx.size + 1, np.int64)
            np.cumsum(lens, out=k_off[1:])
            k_blob = np.frombuffer(b"".join(kb[koff[i]:koff[i + 1]] for i in idx), np.uint8)
        part = {"key_off": k_off, "key_blob": k_blob, "hi": hi[idx], "lo": lo[idx]}
        if is_list:
            ln = loff[idx + 1] - loff[idx]
            l_off = np.zeros(idx.size + 1, np.int64)
            np.cumsum(ln, out=l_off[1:])
            if lcols is not None:
                pidx = np.arange(loff[a], loff[b]) if fix is None else (
                    np.concatenate([np.arange(loff[i], loff[i + 1]) for i in idx]) if idx.size else
                    np.zeros(0, np.int64))
                l_cols = _take_cols(lcols, pidx)
                part.update(list_off=l_off, list_cols=l_cols, val=ln)
                if reducefn is not None:
                    part["py_vals"] = _host_reduce(reducefn, aci, k_off, k_blob, l_off, None, host_values(l_cols))
            else:
                if fix is None:
                    l_val = lval[loff[a]:loff[b]]
                else:
                    l_val = np.concatenate([lval[loff[i]:loff[i + 1]] for i in idx]) if idx.size else lval[:0]
                part.update(list_off=l_off, list_val=l_val, val=ln)
                if reducefn is not None:
                    part["py_vals"] = _host_reduce(reducefn, aci, k_off, k_blob, l_off, l_val)
        else:
            part["cols"] = [c[idx] for c in cols]
            part["val"] = part["cols"][0]
        parts[p] = part
    return parts


def _host_reduce(reducefn, aci: bool, k_off, k_blob, l_off, l_val, vals: list | None = None) -> list:
    """The last resort: the user's reducefn per key over downloaded lists
    (job.lua:264-284; singleton lists skip it under the three ACI flags).
    One host conversion of the partition's values and key bytes, then a
    slice per key (``vals``: the values already as Python objects)."""
    if vals is None:
        vals = l_val.tolist()
    kb = k_blob.tobytes()
    ko = k_off.tolist()
    lo = l_off.tolist()
    out = []
    for i in range(len(ko) - 1):
        values = vals[lo[i]:lo[i + 1]]
        if aci and len(values) == 1:
            out.append(values)
            continue
        o: list = []
        reducefn(codec.key_str(kb[ko[i]:ko[i + 1]]), values, o.append)
        out.append(o)
    return out


# ---------------------------------------------------------------------------
class GenericPlane:
    """The SPMD engine's general plane (``device_reduce`` a column spec, a
    list op with generic emits, or absent)."""

    def __init__(self, eng):
        from .planes import LIST_OPS
        self.eng = eng
        op = eng.op
        self.host_reduce = op is None
        self.unique = op == "concat_unique"
        self.list_mode = op is None or op in LIST_OPS
        # the value row of a posting (parallel/values.py): a number, a tuple
        # of numbers or byte strings
        self.vspec = VL.spec_of(modules.field(eng.mapmod, "device_value_dtype", "i64") or "i64")
        self.dtype = self.vspec if not self.vspec.scalar else self.vspec.dtype
        if not self.list_mode and not self.vspec.scalar:
            raise ValueError(f"device_value_dtype {self.vspec}: tuple and byte-string values go to value lists "
                             "(no device_reduce, 'concat' or 'concat_unique'), not to typed folds")
        self.phys = None if self.list_mode else A.Physical(A.parse_spec(op))
        self._cap = self._cap0 = int(eng.params.get("table_capacity") or 1 << 16)
        red = eng.redmod
        # no device_reduce: the module's own combiner / reducer over the
        # device-grouped lists (batched device hooks, or per key on the host)
        self.reducers = RD.ListReducers(red, self.dtype) if self.host_reduce else None
        self.reducefn = self.reducers.reducefn if self.host_reduce else None
        self.aci = self.reducers.aci if self.host_reduce else False
        self.map = GenericMap(eng.device, self._cap, self.phys, self.dtype, self.reducers,
                              int(eng.params.get("combine_postings") or 0))
        self.red = None
        self._lines = None

    # -- global line numbering (word_lines) ---------------------------------------
    def _line_base(self):
        eng = self.eng
        st = eng.splits
        if st is None:
            return None
        if self._lines is None:
            from .planes import ListPlane
            self._lines = ListPlane.line_offsets(self)  # same all-gather of per-split newline counts

        def base(t):
            a = t.data_ptr() - eng.arena.data_ptr()       # the chunk's offset in the rank's arena
            rel = st.offsets - st.offsets[self._ids0]      # split i starts at rel[i] in the arena
            i = int(np.searchsorted(rel, a, side="right")) - 1
            inside = a - int(rel[i])
            if not inside:
                return int(self._lines[i])
            # newlines of the split before the chunk: counted on the device and
            # added there (no host synchronisation per chunk)
            return torch.count_nonzero(eng.arena[a - inside:a] == 10) + int(self._lines[i])
        return base

    # -- map --------------------------------------------------------------------
    def stream_round_end(self, buf, lo: int, hi: int, heap, H: int) -> None:
        """After a streamed round (SPMDEngine._stage_streaming): the long keys
        the round introduced move their bytes to the key heap at the front of
        the ring buffer, so the round's slot can be refilled (a full heap is
        seen after the map, which then re-runs with a larger one)."""
        self.map.table.rehome_long_keys(buf, lo, hi, heap, H)

    def _issue_ahead(self) -> None:
        f, self._after_issue = getattr(self, "_after_issue", None), None
        if f is not None:
            f()

    def _map_prelude(self, jobs, j0, j1) -> bool:
        """Line numbering and table capacity for a map about to be issued;
        returns whether its input streams through the capped arenas."""
        eng = self.eng
        mp = self.map
        streamed = False
        if eng.device_input == "split" and j1 > j0:
            ids = eng._split_ids(jobs, j0, j1)
            self._ids0 = ids[0]
            streamed = eng._streaming(ids)
        # streamed rounds reuse ring slots: keys are spans of the staged input
        # (rehomed after each round), global line numbers are not available
        mp.emit.line_base = self._line_base() if eng.device_input == "split" and not streamed else None
        if getattr(self, "_table_restored", False) or (mp.table.cap != ops.next_pow2(max(1024, self._cap))
                                                          and mp.table.is_cuda):
            self._table_restored = False
            # the capacity target moved since this table was made (grown, or fitted)
            mp.table = mp.new_table(self._cap)
        return streamed

    def _map_chunks(self, jobs, recs, j0, j1, streamed: bool) -> list:
        """Issue one attempt of the map: every staged chunk through the
        module's device_mapfn (kernels queued, no synchronisation); returns
        the job ranges whose map raised."""
        eng = self.eng
        mp = self.map
        dmap = eng.dmap
        mp.begin(None)
        mp.src.fixed = streamed
        broken = []
        for (a, b), data in eng._stage_chunks(jobs, j0, j1):
            if all(recs[j].status == STATUS.FAILED for j in range(a, b)):
                continue
            if eng.device_input == "split":
                mp.src.set_arena(eng.arena)
            t0, c0 = time.time(), time.process_time()
            for j in range(a, b):
                recs[j].status, recs[j].started, recs[j].worker = STATUS.RUNNING, t0, eng.rank
            mp.emit.chunk = data if isinstance(data, torch.Tensor) and data.dtype == torch.uint8 else None
            keys = [jobs[j][0] for j in range(a, b)]
            try:
                dmap(keys if b - a > 1 else keys[0], data, mp.emit)
                mp.flush_host()
            except (NeedsHostMap, StreamedSourceError):
                raise
            except Exception:  # noqa: BLE001
                mp.host = []
                broken.append((a, b))
                sys.stderr.write("Error executing a job: %s\n" % traceback.format_exc())
            t1 = time.time()
            for j in range(a, b):
                if recs[j].status != STATUS.FAILED:
                    recs[j].status = STATUS.WRITTEN
                recs[j].written = t1
                recs[j].real_time = (t1 - t0) / (b - a)
                recs[j].cpu_time = (time.process_time() - c0) / (b - a)
        return broken

    def _map(self, jobs, recs, j0, j1, issued: tuple | None = None) -> None:
        """The rank's map: issue, synchronise, and re-run on a full table, a
        raising job (BROKEN / FAILED) or a full streaming key heap.
        ``issued``: (streamed, broken) of a first attempt already queued (the
        map the previous iteration issued ahead)."""
        eng = self.eng
        streamed = issued[0] if issued is not None else self._map_prelude(jobs, j0, j1)
        for _attempt in range(64):
            mp = self.map
            if issued is not None and _attempt == 0:
                broken = issued[1]
            else:
                if _attempt:
                    self._map_prelude(jobs, j0, j1)  # (a regrown table)
                broken = self._map_chunks(jobs, recs, j0, j1, streamed)
            self._issue_ahead()  # (before the map's first synchronisation)
            n, ovf = mp.table.stats()
            if streamed and int(ops.host_read(eng._stream_heap)[1]):
                # the key heap ran out: some long keys still point into a ring
                # slot that was refilled — re-map with a heap twice as large
                cur = getattr(eng, "_stream_heap_mb", TUNABLES.stream_heap_mb)
                eng._stream_heap_mb = 2 * cur
                sys.stderr.write("# streaming general map: long-key heap of %.0f MiB full, re-mapping with %.0f MiB\n"
                                 % (cur, 2 * cur))
                continue
            if broken:
                # a chunk whose map raised may have inserted part of its rows:
                # redo the rank's map without it (BROKEN), or leave it out
                # after MAX_JOB_RETRIES attempts (FAILED), server.lua:194-205
                for a, b in broken:
                    for j in range(a, b):
                        recs[j].repetitions += 1
                        recs[j].status = STATUS.FAILED if recs[j].repetitions >= utils.MAX_JOB_RETRIES \
                            else STATUS.BROKEN
                continue
            if ovf or n > mp.table.cap // 2:
                self._cap = ops.next_pow2((16 if ovf else 4) * max(n, 1))  # overflowed: the count is a lower bound
                mp.table = mp.new_table(self._cap)
                continue
            fit = max(ops.next_pow2(2 * max(n, 1)), self._cap0)  # load 1/4 - 1/2
            if n > mp.table.cap // 8 and self._cap < fit:
                self._cap = fit  # next iteration's table
            elif mp.table.cap >= (2 if fit >= _BIG_TABLE else 4) * fit:
                # grown past the key count (4x on a regrowth, 16x after an
                # overflow): fitted for the next maps — large tables from 2x
                # already, their reset and compaction stream every slot (the
                # bigram job's 2^27-slot table: ~2 ms of each step)
                self._cap = fit
            return
        raise RuntimeError("general plane: the map did not converge (table regrowth / retries)")

    # -- pipelined iterations ---------------------------------------------------------
    def _pipelined(self) -> bool:
        """Iteration q+1's map is issued while iteration q reduces (its own
        map state and stream): GPU tables, split inputs prefetched by a pure
        taskfn, no map checkpoints, no streaming."""
        eng = self.eng
        return (bool(eng.pipeline) and eng.device.type == "cuda" and eng._can_pipeline()
                and eng._map_ckpt_path() is None and bool(eng.streams))

    def _map_of(self, q: int) -> "GenericMap":
        """The map state of iteration q when iterations are pipelined (two,
        alternating: the next map fills one while this one is reduced)."""
        if getattr(self, "_maps", None) is None:
            self._maps = [self.map, None]
        m = self._maps[q % 2]
        if m is None:
            m = self._maps[q % 2] = GenericMap(self.eng.device, self._cap, self.phys, self.dtype, self.reducers,
                                               int(self.eng.params.get("combine_postings") or 0))
        return m

    def _issue_next_map(self, jobs, j0, j1, q: int) -> None:
        """Queue iteration q+1's map (same jobs: the taskfn is pure) on its
        own stream and map state; run_iteration(q+1) synchronises it."""
        from .planes import _records
        eng = self.eng
        eng._prefetch(jobs, j0, j1, q + 1)
        cur = self.map
        eng._use(q + 1)
        try:
            with torch.cuda.stream(eng.streams[eng.tslot]):
                self.map = self._map_of(q + 1)
                t0 = time.time()
                recs = _records(eng, jobs, j0, j1, t0)
                streamed = self._map_prelude(jobs, j0, j1)
                broken = self._map_chunks(jobs, recs, j0, j1, streamed)
                nxt = self.map
        finally:
            self.map = cur
            eng._use(q)
        self._pending = {"q": q + 1, "jobs": jobs, "recs": recs, "j0": j0, "j1": j1, "t0": t0, "map": nxt,
                         "issued": (streamed, broken)}

    # -- map checkpoints (split-level restart) ------------------------
    def _save_map(self, recs=None, j0: int = 0, j1: int = 0) -> None:
        """This rank's map output of the iteration -> ``checkpoint_dir``
        (data-only .npz: key words, key bytes, and the physical fold columns or
        the value lists), so a relaunch after a failure later in the iteration
        restores it instead of re-mapping the rank's splits (the fold plane's
        SPMDEngine._save_map for the general plane)."""
        eng = self.eng
        path = eng._map_ckpt_path()
        if path is None:
            return
        import os
        if recs is not None:
            eng._save_job_status(recs, j0, j1)
        mp = self.map
        src = mp.src.source()
        if self.list_mode:
            slot, hi, lo, rep, pslot, pval = mp.table.postings()
        else:
            slot, hi, lo, rep, cols = mp.table.compact()
        _, ln = ops.key_meta(hi, lo, rep, src, want_part=False)
        off, blob = ops.gather_key_bytes(hi, lo, rep, src, lengths=ln)
        arrs = {"hi": hi, "lo": lo, "off": off, "blob": blob,
                "rows": torch.tensor([mp.rows], dtype=torch.int64)}
        if self.list_mode:
            m = hi.numel()
            pos = torch.full((max(self._slot_space(), int(slot.max()) + 1 if m else 1),), -1, dtype=torch.int64,
                             device=slot.device)
            pos[slot] = torch.arange(m, dtype=torch.int64, device=slot.device)
            kidx = pos[pslot.clamp(min=0)]
            keep = (pslot >= 0) & (kidx >= 0)
            arrs["pkey"], arrs["pval"] = kidx[keep], pval[keep]
            if self.vspec.has_bytes:  # byte-string values: their bytes too (row-major over the byte columns)
                arrs["vb_off"], arrs["vb_blob"] = VL.gather_bytes(
                    self.vspec.rows(arrs["pval"])[:, self.vspec.bytes_cols], src)
        else:
            for j, c in enumerate(cols):
                arrs[f"col{j}"] = c
        os.makedirs(eng.checkpoint_dir, exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            np.savez(f, **{k: v.detach().cpu().numpy() for k, v in arrs.items()})
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    def _restore_map(self, recs, j0: int, j1: int) -> bool:
        """Refill the map table from this rank's checkpoint of the iteration,
        if an earlier launch wrote it (the saved keys' bytes become the key
        source); the rank's map jobs are WRITTEN without running."""
        eng = self.eng
        path = eng._map_ckpt_path()
        import os
        if path is None or not os.path.exists(path):
            return False
        with np.load(path, allow_pickle=False) as z:
            a = {k: z[k] for k in z.files}
        d = eng.device
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(d)  # noqa: E731
        koff = a["off"].astype(np.int64)
        lens = np.diff(koff).astype(np.uint64)
        rep = t((((koff[:-1].astype(np.uint64)) << np.uint64(K.REP_LEN_BITS)) | lens).view(np.int64))
        blob = t(np.concatenate([a["blob"], np.zeros(1, np.uint8)]))
        hi, lo = t(a["hi"].view(np.int64)), t(a["lo"].view(np.int64))
        m = hi.numel()
        mp = self.map
        mp.begin(None)
        mp.src.begin(blob)
        cap = ops.next_pow2(max(1 << 12, 4 * m, self._cap))
        if self.list_mode:
            mp.table = mp.new_table(cap)
            kidx = t(a["pkey"])
            pv = t(a["pval"].view(np.int64))
            if self.vspec.has_bytes:
                # the saved value bytes appended to the key source; the span
                # words re-pointed at them
                base = mp.add_bytes(t(a["vb_blob"]))
                rows = self.vspec.rows(pv).clone()
                voff = t(a["vb_off"][:-1].astype(np.int64)).reshape(-1, len(self.vspec.bytes_cols))
                rows[:, self.vspec.bytes_cols] = VL.span_words(
                    voff, VL.word_lengths(rows[:, self.vspec.bytes_cols]), base)
                pv = self.vspec.storage(rows)
            mp.table.src = mp.src.source()
            mp.table.insert(int(kidx.numel()), mp._value_cols(pv), hi=hi[kidx], lo=lo[kidx], rep=rep[kidx])
        else:
            # the saved physical columns are folded 1:1 (the receive side's merge spec)
            merge = [(dt, op, j) for j, (dt, op, _i) in enumerate(self.phys.cols)]
            mp.table = A.AggTable(cap, d, merge)
            mp.table.src = blob
            mp.table.insert(m, [t(a[f"col{j}"]) for j in range(len(merge))], hi=hi, lo=lo, rep=rep)
        self._table_restored = True  # the next map gets a regular table again
        mp.rows = int(a["rows"][0])
        eng._restore_job_status(recs, j0, j1)
        eng.maps_restored += 1
        sys.stderr.write("# rank %d: map of iteration %d restored from its checkpoint\n" % (eng.rank, eng.iteration))
        return True

    # -- shuffle ----------------------------------------------------------------
    def _shuffle(self, keys: tuple, src, failed: int):
        """Send every key (+ folded columns or value list) to rank p % W.
        Returns the received (hi, lo, rep, payload, rblob, failed_total)."""
        eng = self.eng
        W, R = eng.world, eng.nparts
        slot, hi, lo, rep = keys[:4]
        d = hi.device
        m = hi.numel()
        part = devmod.partition_of(hi, lo, rep, src, R, eng.partmod) if m else torch.zeros(0, dtype=torch.int32,
                                                                                           device=d)
        dest = part.to(torch.int64) % W
        kperm = ops.sort_keys_checked([dest], bits=[max(8, _bits(W))]).long() if m else torch.zeros(
            0, dtype=torch.int64, device=d)
        hi, lo, rep, dest, slot = hi[kperm], lo[kperm], rep[kperm], dest[kperm], slot[kperm]
        _, klen = ops.key_meta(hi, lo, rep, src, want_part=False)
        koff, kblob = ops.gather_key_bytes(hi, lo, rep, src, lengths=klen)
        if self.list_mode:
            pslot, pval = keys[4], keys[5]
            pos = torch.full((max(self._slot_space(), 1),), -1, dtype=torch.int64, device=d)
            pos[slot] = torch.arange(m, dtype=torch.int64, device=d)
            pr = pos[pslot.clamp(min=0)]
            ok = (pslot >= 0) & (pr >= 0)
            pr, pv = pr[ok], pval[ok]
            if pr.numel():
                pp = ops.sort_keys_checked([pr], bits=[_bits(m)]).long()
                pr, pv = pr[pp], pv[pp]
            nv = torch.bincount(pr, minlength=m)[:m] if m else torch.zeros(0, dtype=torch.int64, device=d)
            payload = [nv]
            extra = pv
            if self.vspec.has_bytes:
                # byte-string values: their bytes follow the postings (row-
                # major over the byte columns) in one more all-to-all
                bw = self.vspec.rows(pv)[:, self.vspec.bytes_cols]
                vb_off, vb_blob = VL.gather_bytes(bw, src)
                vlen = VL.word_lengths(bw).sum(1)
        else:
            cols = [c[kperm] for c in keys[4]]
            payload = [c.view(torch.int64) if c.dtype == torch.float64 else
                       (c.view(torch.int32).to(torch.int64) if c.dtype == torch.float32 else c) for c in cols]
            nv = None
            extra = None
        cnt = torch.zeros(W, 5, dtype=torch.int64, device=d)
        if m:
            cnt[:, 0].index_add_(0, dest, torch.ones_like(dest))
            cnt[:, 1].index_add_(0, dest, klen.to(torch.int64))
            if nv is not None:
                cnt[:, 2].index_add_(0, dest, nv)
            if extra is not None and self.vspec.has_bytes and pr.numel():
                cnt[:, 4].index_add_(0, dest[pr], vlen)
        cnt[:, 3] = failed
        recv = D.exchange_counts(cnt.view(-1).contiguous(), eng.group).view(W, 5)
        both = torch.cat([cnt, recv]).cpu().tolist()  # one host sync for every split size
        send_c, recv_c = both[:W], both[W:]
        failed_total = sum(r[3] for r in recv_c)
        recs = torch.stack([hi, lo, klen.to(torch.int64)] + payload, 1) if m else torch.zeros(
            (0, 3 + len(payload)), dtype=torch.int64, device=d)
        rrecs = D.all_to_all_v(recs, [c[0] for c in send_c], [c[0] for c in recv_c], eng.group)
        nbytes = sum(c[1] for c in send_c)
        rblob = D.all_to_all_v(kblob[:nbytes], [c[1] for c in send_c], [c[1] for c in recv_c], eng.group)
        rextra = None
        self._rvsrc = None
        if extra is not None:
            rextra = D.all_to_all_v(extra, [c[2] for c in send_c], [c[2] for c in recv_c], eng.group)
            if self.vspec.has_bytes:
                nvb = sum(c[4] for c in send_c)
                rvb = D.all_to_all_v(vb_blob[:nvb], [c[4] for c in send_c], [c[4] for c in recv_c], eng.group)
                # received span words index the sender's source: re-point
                # them at the received value bytes (same row-major order)
                rows = self.vspec.rows(rextra).clone()
                rows[:, self.vspec.bytes_cols] = VL.words_of_lengths(VL.word_lengths(rows[:, self.vspec.bytes_cols]))
                rextra = self.vspec.storage(rows)
                self._rvsrc = rvb if rvb.numel() else torch.zeros(1, dtype=torch.uint8, device=d)
        sent = [32 * c[0] + c[1] + 8 * self.vspec.width * c[2] + c[4] for c in send_c]
        self._nvals_shipped = sum(c[2] for c in send_c) if self.list_mode else sum(c[0] for c in send_c)
        self._shuffled = (sum(sent), sum(sent) - sent[eng.rank])
        rhi, rlo, rlen = rrecs[:, 0].contiguous(), rrecs[:, 1].contiguous(), rrecs[:, 2].contiguous()
        roff, _ = ops.exclusive_scan(rlen)
        rrep = (roff << K.REP_LEN_BITS) | rlen
        if rblob.numel() == 0:
            rblob = torch.zeros(1, dtype=torch.uint8, device=d)
        rpay = [rrecs[:, 3 + j].contiguous() for j in range(len(payload))]
        return rhi, rlo, rrep, rpay, rextra, rblob, failed_total

    def _slot_space(self) -> int:
        t = self.map.table
        return t.cap if t.is_cuda else max(1, t.stats()[0])

    def _merge_received(self, rhi, rlo, rrep, rpay, rextra, rblob):
        """Received keys -> the reduce table (fold: merge the partial columns;
        list: slot per received key, its values in source-rank order)."""
        eng = self.eng
        n = rhi.numel()
        cap = ops.next_pow2(max(1 << 12, 2 * n))
        for _ in range(8):
            if self.list_mode:
                rt = A.AggTable(cap, eng.device, None, "i64")
                rt.src = rblob
                rt.insert(n, [], hi=rhi, lo=rlo, rep=rrep)
            else:
                merge = [(dt, op, j) for j, (dt, op, _i) in enumerate(self.phys.cols)]
                rt = A.AggTable(cap, eng.device, merge)
                rt.src = rblob
                vals = []
                for (dt, _op, _i), c in zip(self.phys.cols, rpay):
                    vals.append(c.view(torch.float64) if dt == "f64" else
                                (c.to(torch.int32).view(torch.float32) if dt == "f32" else c))
                rt.insert(n, vals, hi=rhi, lo=rlo, rep=rrep)
            m, ovf = rt.stats()
            if not ovf and m <= rt.cap // 2 + 1:
                break
            cap *= 4
        else:
            raise OverflowError("reduce table overflow")
        self.red = rt
        if self.list_mode:
            slot, hi, lo, rep, kslot, _ = rt.postings()
            nv = rpay[0]
            pslot = torch.repeat_interleave(kslot, nv, output_size=int(rextra.shape[0]))
            return (slot, hi, lo, rep, pslot, rextra), (rt.cap if rt.is_cuda else max(1, m))
        slot, hi, lo, rep, cols = rt.compact((m, False))
        return (slot, hi, lo, rep, cols), None

    # -- order + reduce (one round, or the rank's partitions in rounds) ---------------
    def _order(self, keys: tuple, src, space, vsrc=None):
        eng = self.eng
        if self.list_mode:
            return order_lists(*keys, src, eng.nparts, eng.partmod, self.unique, self.vspec, space, vsrc=vsrc)
        return order_fold(*keys, src, eng.nparts, eng.partmod, self.phys)

    def _reduce(self, out: dict):
        """The reduce jobs over an ordered result: (device result, None), or
        (None, host partitions) when the module's reducefn ran on the host."""
        R = self.eng.nparts
        if self.host_reduce and self.reducers.device_reduce:
            # batched: device_reducefn over every key's list
            with trace.range("mr.gen.reduce"):
                keys = RD.KeyBatch(out["hi"], out["lo"], key_off=out["key_off"], key_blob=out["key_blob"])
                if "list_cols" in out:
                    red = self.reducers.reduce_device_cols(keys, out["list_off"], out["list_cols"])
                else:
                    red = self.reducers.reduce_device(keys, out["list_off"], out["list_val"])
            out = {k: v for k, v in out.items() if k not in ("list_off", "list_val", "list_cols")}
            out.update(red)
            return out, None
        if self.host_reduce:
            # the last resort: the user's reducefn per key on the host
            return None, host_partitions(out, R, self.vspec, self.reducefn, self.aci)
        return out, None

    def _reduce_groups(self, keys: tuple, src, space):
        """(partition of every key, rounds of partitions) for a reduce under
        reduce_cap_mb — volumes from the key lengths and value counts."""
        from .planes import partition_volumes, reduce_cap_bytes, round_groups
        eng = self.eng
        R = eng.nparts
        hi, lo, rep = keys[1], keys[2], keys[3]
        part, klen = (ops.key_meta(hi, lo, rep, src, nparts=R) if self._fnv_parts() else
                      (devmod.partition_of(hi, lo, rep, src, R, eng.partmod),
                       ops.key_meta(hi, lo, rep, src, want_part=False)[1]))
        if self.list_mode:
            slot, pslot = keys[0], keys[4]
            m = hi.numel()
            pos = torch.full((max(int(space), 1),), -1, dtype=torch.int64, device=hi.device)
            pos[slot] = torch.arange(m, dtype=torch.int64, device=hi.device)
            pr = pos[pslot.clamp(min=0)]
            pr = pr[(pslot >= 0) & (pr >= 0)]
            nv = torch.bincount(pr, minlength=m)[:m] if m else torch.zeros(0, dtype=torch.int64, device=hi.device)
        else:
            nv = torch.full_like(klen, len(keys[4]), dtype=torch.int64)
        vol = partition_volumes(part, klen, nv, R)
        return part, round_groups(vol, reduce_cap_bytes(eng))

    def _fnv_parts(self) -> bool:
        spec = getattr(self.eng.partmod, "device_partition", None) if self.eng.partmod is not None else None
        return spec is not None and spec[0] == "fnv1" and int(spec[1]) == self.eng.nparts

    def _select(self, keys: tuple, space, part, grp: list[int]):
        """The keys (and their values) of partitions ``grp``."""
        km = torch.isin(part.to(torch.int64), torch.tensor(grp, dtype=torch.int64, device=part.device))
        if not self.list_mode:
            slot, hi, lo, rep, cols = keys
            return (slot[km], hi[km], lo[km], rep[km], [c[km] for c in cols]), space
        slot, hi, lo, rep, pslot, pval = keys
        sel = torch.zeros(max(int(space), 1), dtype=torch.bool, device=slot.device)
        sel[slot[km]] = True
        pm = (pslot >= 0) & sel[pslot.clamp(min=0)]
        return (slot[km], hi[km], lo[km], rep[km], pslot[pm], pval[pm]), space

    # -- one iteration --------------------------------------------------------------
    def run_iteration(self, prefetch_next, lookahead):
        eng = self.eng
        eng.iteration += 1
        q = eng._seq
        eng._seq += 1
        eng._use(q)
        pend, self._pending = getattr(self, "_pending", None), None
        if pend is not None and pend["q"] != q:
            pend = None
        pipe = self._pipelined()
        stream = eng.streams[eng.tslot] if (pipe or pend is not None) else None
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            return self._iteration(q, prefetch_next, lookahead, pend, pipe)

    def _iteration(self, q, prefetch_next, lookahead, pend, pipe):
        from .planes import DeviceResult, _records, _result_jobs, reduce_cap_bytes
        eng = self.eng
        res = DeviceResult()
        T = res.timings
        t_start = time.time()
        if pend is not None:  # this iteration's map was queued by the previous one
            jobs, recs, j0, j1, t0 = pend["jobs"], pend["recs"], pend["j0"], pend["j1"], pend["t0"]
            self.map = pend["map"]
        else:
            jobs = eng._jobs()
            j0, j1 = eng._assign(jobs)
            t0 = time.time()
            recs = _records(eng, jobs, j0, j1, t0)
            if pipe:
                self.map = self._map_of(q)
        res.map_jobs = recs
        # the next iterations' input copies (pure taskfn, split inputs) queue
        # right behind this map's, so the copy engine streams while this
        # iteration reduces: its arena was last read by iteration q - 2 or
        # earlier, whose key bytes were gathered (and synchronised) by its order
        ahead = 0 if not (prefetch_next if prefetch_next is not None else eng.prefetch) else (
            2 if lookahead is None else min(lookahead, 2))
        self._after_issue = (lambda: eng._prefetch_ahead(jobs, j0, j1, q, ahead)) if ahead else None
        # iteration q+1's map is queued once this iteration's order is (it runs
        # on its own stream while this one's tail and downloads finish)
        next_map = [pipe and ahead > 0]

        def issue_next_map():
            if next_map[0]:
                next_map[0] = False
                with trace.range("mr.gen.issue_next"):
                    self._issue_next_map(jobs, j0, j1, q)
        with trace.range("mr.gen.map"):
            if pend is not None:
                self._map(jobs, recs, j0, j1, issued=pend["issued"])
                self.map.combine()
                self._save_map(recs, j0, j1)
            elif not self._restore_map(recs, j0, j1):
                self._map(jobs, recs, j0, j1)
                self.map.combine()  # the end-of-map combiner (job.lua:198-202); no-op without one
                self._save_map(recs, j0, j1)
            self._issue_ahead()
        eng._maybe_inject_fault("shuffle")
        T["map"] = time.time() - t0
        t1 = time.time()
        mp = self.map
        src = mp.src.source()
        R, W = eng.nparts, eng.world
        failed = sum(1 for r in recs[j0:j1] if r.status == STATUS.FAILED)
        if self.list_mode:
            keys = mp.table.postings()
            space = self._slot_space()
        else:
            keys = mp.table.compact()
            space = None
        self._shuffled = (0, 0)
        self._nvals_shipped = 0
        res.distinct_keys_map = int(keys[1].numel())
        vsrc = src  # byte-string values: spans of the key source until the shuffle moves them
        if W > 1 or eng.force_shuffle:
            with trace.range("mr.gen.shuffle"):
                rhi, rlo, rrep, rpay, rextra, rblob, failed = self._shuffle(keys, src, failed)
                keys, space = self._merge_received(rhi, rlo, rrep, rpay, rextra, rblob)
                src = rblob
                vsrc = self._rvsrc if self._rvsrc is not None else rblob
        T["shuffle"] = time.time() - t1
        t2 = time.time()
        res.total_value = mp.rows
        res.failed_maps = failed
        res.bytes_shuffled, res.bytes_shuffled_remote = self._shuffled
        groups = self._reduce_groups(keys, src, space) if reduce_cap_bytes(eng) else None
        c0 = time.process_time()
        if groups is not None and len(groups[1]) > 1:
            # reduce-side out-of-core (the reference's reduce streams its
            # inputs, utils.lua:133-271): the rank's partitions in rounds of at
            # most reduce_cap_mb, each ordered and reduced on the device and
            # moved to host memory before the next
            part, rounds = groups
            parts, counts, nk = {}, [0] * R, 0
            issue_next_map()
            for grp in rounds:
                sub, sub_space = self._select(keys, space, part, grp)
                with trace.range("mr.gen.order"):
                    out = self._order(sub, src, sub_space, vsrc)
                counts = [a + b for a, b in zip(counts, out["counts"].cpu().tolist())]
                nk += int(out["hi"].numel())
                dev_out, got = self._reduce(out)
                parts.update(got if got is not None else host_partitions(dev_out, R, self.vspec))
                del out, dev_out, sub
            self.reduce_rounds = len(rounds)
            _result_jobs(eng, res, counts, t1)
            res.device = None
            res._parts = parts
            res.distinct_keys = nk
        else:
            with trace.range("mr.gen.order"):
                out = self._order(keys, src, space, vsrc)
                issue_next_map()
                counts = out["counts"].cpu().tolist()
            self.reduce_rounds = 1
            _result_jobs(eng, res, counts, t1)
            res.distinct_keys = int(out["hi"].numel())
            dev_out, parts = self._reduce(out)
            res.device = dev_out
            if parts is not None:
                res._parts = parts
            else:
                res._materialize = lambda o=dev_out: host_partitions(o, R, self.vspec)
        if self.host_reduce and not self.reducers.device_reduce:
            cpu = time.process_time() - c0
            parts = res._parts or {}
            for r in res.red_jobs:
                r.cpu_time = cpu * len(parts.get(int(r.key), {}).get("py_vals", [])) / max(1, res.distinct_keys)
        T["reduce"] = time.time() - t2
        T["iteration"] = time.time() - t_start
        return res
