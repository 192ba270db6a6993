"""Group-by on a CSV column with float aggregates, as a MapReduce job: input
lines ``word,score``; result per word = [mean score, max score, count].  The
device map emits every line as (word span, score, score, 1) with
``emit.csv`` (one fused GPU kernel: line and field split, decimal parse and
the LDS-combined typed fold; specified by ops/text.py csv_rows); the reduce module's
``device_reduce = ("f64:mean", "f64:max", "count")`` folds them in typed
columns of the general plane (native f64 atomics; a mean is kept as a sum
and a count and divided when results are read).  The host ``reducefn``
computes the same list from the raw scores (server/worker host plane, the
oracle), the way the reference's reducers fold a value list
(/root/reference/mapreduce/job.lua:98-106,264-284).

* ``taskfn``: one map job per split (``init({"nsplits": N})``, SPMD staged
  splits) or per file (``init({"files": [...]})``).
* partition: FNV-1 of the word mod R.
* finalfn: the per-word lists in ``RESULT`` unless ``{"quiet": true}``.
"""
from __future__ import annotations

NUM_REDUCERS = 6
NSPLITS = 4
FILES: list[str] = []
QUIET = False
RESULT: dict = {}


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


def device_mapfn(key, value, emit):
    if hasattr(value, "data_ptr"):
        data = value
    else:
        from lua_mapreduce_1_amd.ops import io as _io
        data = _io.load_file(value["file"] if isinstance(value, dict) else value, emit.device)
    # key = field 0, inputs (score, score, 1); rows without a valid score
    # emit nothing.  On the GPU one fused kernel (lines, fields, parse, the
    # LDS-combined fold); its specification is the ops/text.py chain
    # TX.csv_rows (lines -> field -> parse_f64).
    emit.csv(data, key=0, values=(1, 1, None), sep=",")


def _rows(data: bytes):
    for line in data.split(b"\n"):
        if line.endswith(b"\r"):
            line = line[:-1]
        parts = line.split(b",")
        if len(parts) < 2 or not parts[0]:
            continue
        try:
            v = float(parts[1].decode("ascii").strip())
        except ValueError:
            continue
        yield parts[0].decode("utf-8", "surrogateescape"), v


def mapfn(key, value, emit):
    with open(value["file"] if isinstance(value, dict) else value, "rb") as f:
        for k, v in _rows(f.read()):
            emit(k, v)


device_partition = ("fnv1", NUM_REDUCERS)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    emit(sum(values) / len(values))
    emit(max(values))
    emit(len(values))


device_reduce = ("f64:mean", "f64:max", "count")


def finalfn(pairs_iterator):
    global RESULT
    out = {}
    for key, values in pairs_iterator:
        out[key] = list(values)
    RESULT = {} if QUIET else out
    return True


def naive(splits: list[bytes]) -> dict:
    """Oracle: word -> [mean, max, count]."""
    acc: dict = {}
    for s in splits:
        for k, v in _rows(s):
            acc.setdefault(k, []).append(v)
    return {k: [sum(v) / len(v), max(v), len(v)] for k, v in acc.items()}
