"""Data-only codecs for intermediate (``map_results.P<p>.M<m>``) and result
(``result.P<NN>``) files.

The reference writes executable Lua lines ``return k,{v1,...}`` and reads
them back with ``load(line)()`` (job.lua:212-214, utils.lua:222-224,
server.lua:380-382) — code execution on the data path.  Two data-only formats
replace it:

* ``MRK1`` — msgpack stream of ``[key, [values...]]`` records in key order
  (host plane: arbitrary Python keys/values from user map/reduce functions).
* ``MRC1`` — columnar device format: u64 key words (hi, lo), int64 values and
  the key bytes (offsets + blob), straight from HBM buffers (device plane);
  ``MRC2`` the same with K typed value columns (the general plane's folds).
"""
from __future__ import annotations

import struct
from typing import Iterable, Iterator

import msgpack
import numpy as np

MAGIC_REC = b"MRK1"
MAGIC_COL = b"MRC1"


def _default(o):
    if isinstance(o, (set, frozenset)):
        return list(o)
    if isinstance(o, np.integer):
        return int(o)
    if isinstance(o, np.floating):
        return float(o)
    raise TypeError(f"cannot serialize {type(o).__name__}")


def encode_records(records: Iterable[tuple]) -> bytes:
    # keys from byte data are str with surrogate escapes (non-UTF-8 bytes,
    # key_str): packed as such and decoded with the same handler, so any
    # byte string round-trips (the reference's keys are arbitrary Lua strings)
    pk = msgpack.Packer(use_bin_type=True, default=_default, unicode_errors="surrogateescape")
    out = [MAGIC_REC]
    for k, vals in records:
        out.append(pk.pack([k, list(vals)]))
    return b"".join(out)


def _fix(x):
    # msgpack arrays decode as tuples (use_list=False): keep tuples for keys
    # (hashable, like the reference's interned tuples) and values.
    return x


def decode_records(data: bytes) -> Iterator[tuple]:
    if not data:
        return iter(())
    if data[:4] == MAGIC_COL:
        return iter_columnar(decode_columnar(data))
    if data[:4] == MAGIC_COL2:
        return iter_columnar(decode_columns(data))
    if data[:4] != MAGIC_REC:
        raise ValueError("unknown intermediate file format")
    up = msgpack.Unpacker(use_list=False, raw=False, strict_map_key=False, unicode_errors="surrogateescape")
    up.feed(memoryview(data)[4:])
    return ((k, list(v)) for k, v in up)


# ---------------------------------------------------------------------------
def encode_columnar(hi: np.ndarray, lo: np.ndarray, val: np.ndarray, key_off: np.ndarray,
                    key_blob: np.ndarray) -> bytes:
    n = int(hi.size)
    nb = int(key_blob.size)
    head = MAGIC_COL + struct.pack("<QQ", n, nb)
    return b"".join([head, np.ascontiguousarray(hi, np.uint64).tobytes(), np.ascontiguousarray(lo, np.uint64).tobytes(),
                     np.ascontiguousarray(val, np.int64).tobytes(), np.ascontiguousarray(key_off, np.int64).tobytes(),
                     np.ascontiguousarray(key_blob, np.uint8).tobytes()])


def decode_columnar(data: bytes) -> dict:
    if data[:4] != MAGIC_COL:
        raise ValueError("not a columnar file")
    n, nb = struct.unpack("<QQ", data[4:20])
    p = 20
    out = {}
    for name, dt, cnt in (("hi", np.uint64, n), ("lo", np.uint64, n), ("val", np.int64, n),
                          ("key_off", np.int64, n + 1), ("key_blob", np.uint8, nb)):
        sz = np.dtype(dt).itemsize * cnt
        out[name] = np.frombuffer(data, dtype=dt, count=cnt, offset=p)
        p += sz
    return out


# ---------------------------------------------------------------------------
MAGIC_COL2 = b"MRC2"
_DT_CODE = {np.dtype(np.int64): 0, np.dtype(np.float64): 1, np.dtype(np.float32): 2}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}


def encode_columns(hi: np.ndarray, lo: np.ndarray, cols: list, key_off: np.ndarray, key_blob: np.ndarray) -> bytes:
    """``MRC2``: keys + K typed value columns (int64 / float64 / float32),
    the general plane's folds (parallel/generic.py)."""
    n, nb, k = int(hi.size), int(key_blob.size), len(cols)
    codes = bytes(_DT_CODE[np.asarray(c).dtype] for c in cols).ljust(8 * ((k + 7) // 8), b"\0")
    parts = [MAGIC_COL2, struct.pack("<QQQ", n, nb, k), codes, np.ascontiguousarray(hi, np.uint64).tobytes(),
             np.ascontiguousarray(lo, np.uint64).tobytes(), np.ascontiguousarray(key_off, np.int64).tobytes()]
    parts += [np.ascontiguousarray(c).tobytes() for c in cols]
    parts.append(np.ascontiguousarray(key_blob, np.uint8).tobytes())
    return b"".join(parts)


def decode_columns(data: bytes) -> dict:
    if data[:4] != MAGIC_COL2:
        raise ValueError("not an MRC2 file")
    n, nb, k = struct.unpack("<QQQ", data[4:28])
    p = 28
    codes = data[p:p + k]
    p += 8 * ((k + 7) // 8)
    out = {}
    for name, cnt in (("hi", n), ("lo", n)):
        out[name] = np.frombuffer(data, dtype=np.uint64, count=cnt, offset=p)
        p += 8 * cnt
    out["key_off"] = np.frombuffer(data, dtype=np.int64, count=n + 1, offset=p)
    p += 8 * (n + 1)
    cols = []
    for c in codes:
        dt = _CODE_DT[c]
        cols.append(np.frombuffer(data, dtype=dt, count=n, offset=p))
        p += dt.itemsize * n
    out["cols"] = cols
    out["key_blob"] = np.frombuffer(data, dtype=np.uint8, count=nb, offset=p)
    return out


def key_str(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def iter_columnar(cols: dict) -> Iterator[tuple]:
    """(key, values) pairs of a device result partition: one folded value per
    key (``val``), a value list per key (``list_off`` / ``list_val``, the list
    plane), or fixed-width records (``records`` with ``key_bytes``: key = the
    record's key bytes, value = the rest of the record as bytes)."""
    if "records" in cols:
        rec = cols["records"]
        kb = int(cols["key_bytes"])
        for i in range(int(rec.shape[0])):
            row = rec[i].tobytes()
            yield key_str(row[:kb]), [row[kb:]]
        return
    off = cols["key_off"]
    blob = cols["key_blob"].tobytes()
    if "py_vals" in cols:  # a host reducefn's output per key (parallel/generic.py)
        for i, v in enumerate(cols["py_vals"]):
            yield key_str(blob[off[i]:off[i + 1]]), list(v)
        return
    if "cols" in cols:  # typed fold columns: one value per column
        cs = cols["cols"]
        for i in range(int(off.size) - 1):
            yield key_str(blob[off[i]:off[i + 1]]), [c[i].item() for c in cs]
        return
    if "list_cols" in cols:  # tuple / byte-string values (parallel/values.py): (off, blob) per byte column
        lo = cols["list_off"]
        py = []
        for c in cols["list_cols"]:
            if isinstance(c, tuple):
                o, b = c[0], c[1].tobytes()
                py.append([key_str(b[o[i]:o[i + 1]]) for i in range(len(o) - 1)])
            else:
                py.append(c.tolist())
        vals = py[0] if len(py) == 1 else list(zip(*py))
        for i in range(int(lo.size) - 1):
            yield key_str(blob[off[i]:off[i + 1]]), vals[lo[i]:lo[i + 1]]
        return
    if "list_off" in cols:
        lo, lv = cols["list_off"], cols["list_val"]
        for i in range(int(lo.size) - 1):
            yield key_str(blob[off[i]:off[i + 1]]), lv[lo[i]:lo[i + 1]].tolist()
        return
    val = cols["val"]
    for i in range(int(val.size)):
        yield key_str(blob[off[i]:off[i + 1]]), [int(val[i])]
