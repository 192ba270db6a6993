"""Per-endpoint latency percentiles as a MapReduce job — a reducer that no
built-in fold expresses (a quantile needs the whole value list), run on the
GPU through the batched ``device_reducefn`` hook.

Input lines ``endpoint,latency_ms``.  Result per endpoint:
[p50, p90, p99, max, count] (percentiles linearly interpolated between the
sorted values, as numpy's default).  The reference runs such a reducer per
key in Lua over the grouped values (/root/reference/mapreduce/job.lua:264-284);
here ``reducefn`` is that per-key form (server/worker host plane, the oracle)
and ``device_reducefn`` the same reducer over every key's list at once: one
segmented sort of all lists (ops/segments.py) and gathers at the percentile
positions.  There is no combiner (a percentile does not combine), so every
value is shipped to its reducer, as the reference does without one.

* ``device_mapfn``: ``emit.csv`` — key field 0, value field 1 (float64
  values: ``device_value_dtype = "f64"``); rows whose latency does not parse
  are dropped.
* partition: FNV-1 of the endpoint mod R.
"""
from __future__ import annotations

import math

NUM_REDUCERS = 6
NSPLITS = 4
FILES: list[str] = []
QUIET = False
RESULT: dict = {}
QS = (0.5, 0.9, 0.99)


def init(args):
    global NUM_REDUCERS, NSPLITS, FILES, QUIET, device_partition
    if isinstance(args, dict):
        NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
        FILES = list(args.get("files") or [])
        NSPLITS = int(args.get("nsplits", len(FILES) or NSPLITS))
        QUIET = bool(args.get("quiet", False))
    device_partition = ("fnv1", NUM_REDUCERS)


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"file": FILES[i], "split": i} if FILES else {"split": i})


spmd_replicated_taskfn = True
device_input = "split"
device_value_dtype = "f64"
device_partition = ("fnv1", NUM_REDUCERS)


def device_mapfn(key, value, emit):
    if hasattr(value, "data_ptr"):
        data = value
    else:
        from lua_mapreduce_1_amd.ops import io as _io
        data = _io.load_file(value["file"] if isinstance(value, dict) else value, emit.device)
    emit.csv(data, key=0, values=(1,), sep=",")


def _rows(data: bytes):
    for line in data.split(b"\n"):
        if line.endswith(b"\r"):
            line = line[:-1]
        f = line.split(b",")
        if len(f) < 2 or not f[0]:
            continue
        try:
            v = float(f[1])
        except ValueError:
            continue
        yield f[0].decode("utf-8", "surrogateescape"), v


def mapfn(key, value, emit):
    with open(value["file"] if isinstance(value, dict) else value, "rb") as f:
        data = f.read()
    for k, v in _rows(data):
        emit(k, v)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def _percentile(sv: list, q: float) -> float:
    pos = (len(sv) - 1) * q
    lo, hi = math.floor(pos), math.ceil(pos)
    return sv[lo] + (sv[hi] - sv[lo]) * (pos - lo)


def reducefn(key, values, emit):
    sv = sorted(values)
    for q in QS:
        emit(_percentile(sv, q))
    emit(sv[-1])
    emit(len(sv))


def device_reducefn(keys, off, val):
    """Every key's [p50, p90, p99, max, count] at once: one segmented sort of
    all value lists, then gathers at the interpolation positions."""
    import torch
    from lua_mapreduce_1_amd.ops import segments as S
    ln = S.lengths(off)
    sv = S.sort(off, val).to(torch.float64)
    last = (off[1:] - 1).clamp(min=0)
    cols = []
    for q in QS:
        pos = (ln - 1).clamp(min=0).to(torch.float64) * q
        lo = pos.floor().to(torch.int64)
        hi = pos.ceil().to(torch.int64)
        a, b = sv[off[:-1] + lo], sv[off[:-1] + hi]
        cols.append(a + (b - a) * (pos - lo.to(torch.float64)))
    cols.append(sv[last])
    cols.append(ln.to(torch.float64))
    return torch.stack(cols, dim=1)


def finalfn(pairs_iterator):
    global RESULT
    RESULT = {k: list(v) for k, v in pairs_iterator}
    if not QUIET:
        print("# endpoints:", len(RESULT))
    return True


def make_log(seed: int = 0, lines: int = 100_000, endpoints: int = 200, nsplits: int = 4) -> list[bytes]:
    """Synthetic access-log lines ``/api/endpoint_<k>,<latency ms>``: Zipf
    endpoint popularity, log-normal latencies with a per-endpoint scale, a few
    malformed latencies (dropped by the map)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, endpoints + 1)
    ep = rng.choice(endpoints, size=lines, p=w / w.sum())
    scale = rng.uniform(1.0, 50.0, endpoints)
    lat = np.round(rng.lognormal(0.0, 0.7, lines) * scale[ep], 3)
    out = []
    per = -(-lines // nsplits)
    for s in range(nsplits):
        rows = []
        for i in range(s * per, min(lines, (s + 1) * per)):
            v = "n/a" if i % 997 == 13 else "%.3f" % lat[i]
            rows.append("/api/endpoint_%d,%s\n" % (ep[i], v))
        out.append("".join(rows).encode())
    return out


def naive(splits: list[bytes]) -> dict:
    acc: dict = {}
    for s in splits:
        for k, v in _rows(s):
            acc.setdefault(k, []).append(v)
    out = {}
    for k, vs in acc.items():
        res: list = []
        reducefn(k, vs, res.append)
        out[k] = res
    return out
