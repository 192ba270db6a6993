"""Value rows of the general device plane's value lists: numbers, fixed-width
tuples and byte strings.

The reference wraps every emitted value in ``tuple(value)``
(/root/reference/mapreduce/job.lua:84) and serialises strings and tables into
its intermediate files (utils.lua:100-120, job.lua:212-214), so a mapper may
emit a number, a string, or a small table per key — the APRIL-ANN example
emits serialised byte blobs (examples/APRIL-ANN/common.lua:95-103).  Here a
posting (one emitted value) is a row of ``k`` 8-byte words, declared by the
map module's ``device_value_dtype``:

* ``"i64"`` / ``"f64"`` — one number (the original value lists);
* a tuple such as ``("i64", "i64")`` or ``("i64", "f64")`` — a k-tuple of
  numbers (e.g. a (document, position) posting);
* ``"bytes"`` (also inside a tuple) — a byte string, stored as a span word
  ``offset << 24 | length`` into the plane's byte source (the staged input the
  map reads, or bytes appended to it), like the keys' rep words.  Its bytes
  travel with the shuffle and come back as ``str`` (surrogate-escaped, as
  keys do).

Device hooks (``device_combinerfn`` / ``device_reducefn``) receive the values
of a width-1 numeric list as a tensor [n], of byte strings as a
:class:`ByteValues` (CSR of the bytes), of a numeric tuple with one dtype as a
tensor [n, k], and otherwise as a tuple of per-column values: a typed tensor
[n] per number column, a ByteValues per byte column.
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch

from ..ops import keys as K

TYPES = ("i64", "f64", "bytes")
_LONG_MARK = 0xFF


class ByteValues(NamedTuple):
    """Byte-string values in CSR form: value i = ``blob[off[i]:off[i + 1]]``."""
    off: torch.Tensor
    blob: torch.Tensor

    def strings(self) -> list[str]:
        o = self.off.cpu().numpy()
        b = self.blob.cpu().numpy().tobytes()
        return [b[o[i]:o[i + 1]].decode("utf-8", "surrogateescape") for i in range(o.size - 1)]


class ByteSpans(NamedTuple):
    """An emitted byte-string value column: value i = ``text[starts[i] :
    starts[i] + lens[i]]`` (``text`` None: the chunk being mapped)."""
    starts: torch.Tensor
    lens: torch.Tensor
    text: torch.Tensor | None = None


class ValueSpec:
    """The value row of a list-mode plane (see the module docstring)."""

    def __init__(self, spec="i64"):
        if isinstance(spec, ValueSpec):
            spec = spec.cols
        cols = (str(spec),) if isinstance(spec, str) else tuple(str(c) for c in spec)
        if not cols or any(c not in TYPES for c in cols):
            raise ValueError(f"device_value_dtype: 'i64', 'f64', 'bytes' or a tuple of them (got {spec!r})")
        if len(cols) > 8:
            raise ValueError("device_value_dtype: at most 8 value columns")
        self.cols = cols
        self.width = len(cols)
        self.bytes_cols = [j for j, c in enumerate(cols) if c == "bytes"]
        # the original value lists: one number per posting, 1-D storage
        self.scalar = self.width == 1 and not self.bytes_cols

    @property
    def dtype(self) -> str:
        """The number dtype of a scalar spec ('i64' / 'f64'), else 'tuple'."""
        return self.cols[0] if self.scalar else "tuple"

    @property
    def has_bytes(self) -> bool:
        return bool(self.bytes_cols)

    def __eq__(self, o) -> bool:
        return isinstance(o, ValueSpec) and o.cols == self.cols

    def __repr__(self) -> str:
        return f"ValueSpec({self.cols if self.width > 1 else self.cols[0]!r})"

    def rows(self, bits: torch.Tensor) -> torch.Tensor:
        """Posting storage as [n, k] (a scalar spec's 1-D storage viewed)."""
        return bits.reshape(-1, self.width)

    def storage(self, rows: torch.Tensor) -> torch.Tensor:
        """[n, k] rows -> the plane's storage (1-D for a scalar spec)."""
        return rows.reshape(-1) if self.scalar else rows.reshape(-1, self.width)


def spec_of(dtype) -> ValueSpec:
    return dtype if isinstance(dtype, ValueSpec) else ValueSpec(dtype or "i64")


# -- byte-string values ----------------------------------------------------------
def span_words(starts: torch.Tensor, lens: torch.Tensor, base: int) -> torch.Tensor:
    """Span words ``(base + start) << 24 | len`` of byte values."""
    st = starts.to(torch.int64)
    ln = lens.to(torch.int64).clamp(min=0, max=K.REP_LEN_MASK)
    return ((st + int(base)) << K.REP_LEN_BITS) | ln


def word_lengths(words: torch.Tensor) -> torch.Tensor:
    return words & K.REP_LEN_MASK


def gather_bytes(words: torch.Tensor, src: torch.Tensor):
    """Bytes of span words (any shape, taken in row-major order) -> CSR
    (off int64 [n + 1], blob uint8) — one gather launch on the GPU (the
    key-byte gather, every value read as a long key through its span)."""
    from .. import ops
    w = words.reshape(-1).contiguous()
    n = w.numel()
    d = w.device
    if n == 0:
        return torch.zeros(1, dtype=torch.int64, device=d), torch.zeros(0, dtype=torch.uint8, device=d)
    z = torch.zeros(n, dtype=torch.int64, device=d)
    mark = torch.full((n,), _LONG_MARK, dtype=torch.int64, device=d)
    lens = word_lengths(w)
    return ops.gather_key_bytes(z, mark, w, src, lengths=lens)


def words_of_lengths(lens: torch.Tensor) -> torch.Tensor:
    """Span words of values laid out back to back (offsets = exclusive scan of
    the lengths): the received value bytes of a shuffle."""
    from .. import ops
    ln = lens.reshape(-1).to(torch.int64).contiguous()
    off, _ = ops.exclusive_scan(ln) if ln.numel() else (ln, None)
    return ((off << K.REP_LEN_BITS) | ln).reshape(lens.shape)


def byte_values(words: torch.Tensor, src: torch.Tensor) -> ByteValues:
    off, blob = gather_bytes(words, src)
    return ByteValues(off, blob)


# -- the values device hooks see -------------------------------------------------------
def _typed(bits: torch.Tensor, dt: str) -> torch.Tensor:
    return bits.view(torch.float64) if dt == "f64" else bits


def to_user(bits: torch.Tensor, spec: ValueSpec, src: torch.Tensor | None):
    """Stored posting bits -> the values a device hook receives."""
    if spec.scalar:
        return _typed(bits, spec.cols[0])
    rows = spec.rows(bits)
    if spec.width == 1:  # one byte-string column
        return byte_values(rows[:, 0].contiguous(), src)
    if not spec.has_bytes and len(set(spec.cols)) == 1:
        return _typed(rows.contiguous(), spec.cols[0])
    out = []
    for j, c in enumerate(spec.cols):
        col = rows[:, j].contiguous()
        out.append(byte_values(col, src) if c == "bytes" else _typed(col, c))
    return tuple(out)


def from_user(vals, spec: ValueSpec, n: int, add_bytes, who: str) -> torch.Tensor:
    """A hook's returned values (the same forms as :func:`to_user`, n rows)
    -> storage bits; byte values are appended to the byte source through
    ``add_bytes(uint8 tensor) -> offset``."""
    if spec.scalar:
        from .reducers import _bits, _to_list_dtype
        return _bits(_to_list_dtype(vals, spec.cols[0], who))
    if isinstance(vals, ByteValues):
        vals = (vals,)
    if isinstance(vals, torch.Tensor):
        if vals.dim() != 2 or vals.shape[1] != spec.width or spec.has_bytes:
            raise ValueError(f"{who}: values of {spec} must come back as [n, {spec.width}] (or a tuple of columns)")
        cols = [vals[:, j] for j in range(spec.width)]
    else:
        cols = list(vals)
        if len(cols) != spec.width:
            raise ValueError(f"{who}: {len(cols)} value columns returned, {spec} has {spec.width}")
    outs = []
    for c, dt in zip(cols, spec.cols):
        if dt == "bytes":
            if not isinstance(c, ByteValues):
                raise TypeError(f"{who}: a byte-string value column must come back as ByteValues(off, blob)")
            base = add_bytes(c.blob.to(torch.uint8))
            outs.append(span_words(c.off[:-1], c.off[1:] - c.off[:-1], base))
        else:
            from .reducers import _bits, _to_list_dtype
            outs.append(_bits(_to_list_dtype(c.reshape(-1), dt, who)))
    if any(o.numel() != n for o in outs):
        raise ValueError(f"{who}: every value column needs {n} rows")
    return torch.stack(outs, 1) if outs else torch.zeros((n, 0), dtype=torch.int64)


# -- host values (results, host reducefn / combinerfn) -------------------------------------
def host_columns(bits: np.ndarray, spec: ValueSpec, byte_csr: dict | None = None) -> list:
    """Stored posting bits (host numpy) -> one Python value per posting: a
    number, a str, or a tuple of them.  ``byte_csr``: {column: (off, blob)} of
    the byte columns, in posting order."""
    if spec.scalar:
        v = bits.view(np.float64) if spec.cols[0] == "f64" else bits
        return v.tolist()
    rows = bits.reshape(-1, spec.width)
    cols = []
    for j, c in enumerate(spec.cols):
        col = np.ascontiguousarray(rows[:, j])
        if c == "bytes":
            off, blob = byte_csr[j]
            b = blob.tobytes()
            cols.append([b[off[i]:off[i + 1]].decode("utf-8", "surrogateescape") for i in range(off.size - 1)])
        else:
            cols.append((col.view(np.float64) if c == "f64" else col).tolist())
    if spec.width == 1:
        return cols[0]
    return list(zip(*cols))


def host_bits(values: list, spec: ValueSpec, add_bytes, who: str) -> np.ndarray:
    """Python values (numbers / strings / tuples, one per posting) -> storage
    bits (numpy int64 [n] or [n, k]); strings are appended to the byte source
    through ``add_bytes(bytes) -> offset``."""
    n = len(values)
    rows = [v if isinstance(v, (tuple, list)) else (v,) for v in values] if not spec.scalar else None
    if spec.scalar:
        dt = spec.cols[0]
        try:
            arr = np.asarray(values, dtype=np.float64 if dt == "f64" else None)
        except (TypeError, ValueError) as e:
            raise TypeError(f"{who} emitted values that are not numbers: {e}") from None
        if arr.size and dt == "i64":
            if arr.dtype.kind == "f" and not np.all(np.floor(arr) == arr):
                raise TypeError(f"{who} emitted {arr.dtype} values into i64 value lists (declare "
                                "device_value_dtype = 'f64' on the map module for real values)")
            if arr.dtype.kind not in "iubf":
                raise TypeError(f"{who} emitted values that are not numbers")
            arr = arr.astype(np.int64)
        arr = arr.astype(np.float64 if dt == "f64" else np.int64, copy=False).reshape(n)
        return arr.view(np.int64) if dt == "f64" else arr
    out = np.zeros((n, spec.width), np.int64)
    for i, r in enumerate(rows):
        if len(r) != spec.width:
            raise TypeError(f"{who} emitted a value of {len(r)} fields into {spec} value lists")
    for j, dt in enumerate(spec.cols):
        col = [r[j] for r in rows]
        if dt == "bytes":
            bs = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x) for x in col]
            base = add_bytes(b"".join(bs)) if bs else 0
            lens = np.array([len(b) for b in bs], np.int64)
            starts = np.zeros(n, np.int64)
            if n:
                np.cumsum(lens[:-1], out=starts[1:])
            out[:, j] = ((starts + base) << K.REP_LEN_BITS) | lens
        elif dt == "f64":
            out[:, j] = np.asarray(col, np.float64).view(np.int64)
        else:
            a = np.asarray(col)
            if a.size and a.dtype.kind == "f" and not np.all(np.floor(a) == a):
                raise TypeError(f"{who} emitted real values into an i64 value column")
            out[:, j] = a.astype(np.int64)
    return out


def order_words(rows: torch.Tensor, spec: ValueSpec) -> list[torch.Tensor]:
    """int64 words whose unsigned lexicographic order is the numeric order of
    numeric value rows (for concat_unique over tuples)."""
    sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=rows.device)
    out = []
    for j, dt in enumerate(spec.cols):
        v = rows[:, j]
        out.append(torch.where(v < 0, ~v, v ^ sign) if dt == "f64" else v ^ sign)
    return out
