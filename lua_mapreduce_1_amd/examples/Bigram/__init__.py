"""Bigram count as a MapReduce job: every pair of consecutive whitespace
tokens on one line -> number of occurrences.  The key of a pair is the byte
span from the first token's start to the second token's end (``"w1 w2"``
for single-spaced text), so keys are not tokens of the input: the device map
picks them with ops/text.py (``ngrams``) and emits byte spans
(``emit.spans``), which the int64 fold plane sums like word counts.  One
module holds every function, like the reference's single-module WordCount
(/root/reference/mapreduce/examples/WordCount/init.lua).

* ``taskfn``: one map job per split — ``init({"nsplits": N})`` for splits
  staged by the SPMD engine (``device_input = "split"``), or
  ``init({"files": [...]})`` (server/worker, host SPMD plane): each job value
  carries its file.
* partition: exact FNV-1 of the key mod R (examples/WordCount/partitionfn.lua).
* reduce: sum, also the combiner; associative/commutative/idempotent.
* finalfn: the counts in ``RESULT`` unless ``{"quiet": true}``.
"""
from __future__ import annotations

import re

NUM_REDUCERS = 8
NSPLITS = 4
FILES: list[str] = []
QUIET = False
RESULT: dict = {}
_TOKEN = re.compile(rb"[^ \t\n\v\f\r]+")


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


def _data(value, emit):
    if hasattr(value, "data_ptr"):
        return value  # SPMD: the staged split(s)
    from lua_mapreduce_1_amd.ops import io as _io
    return _io.load_file(value["file"] if isinstance(value, dict) else value, emit.device)


def device_mapfn(key, value, emit):
    from lua_mapreduce_1_amd.ops import text as TX
    data = _data(value, emit)
    # every token with the span to the end of the next token on its line
    # (length 0 at a line's last token: emit.spans skips it) — one pass over
    # the bytes; the same as tokens(lines=True) + torch ops pairing token i
    # with token i+1 where both lines agree (see ops/text.py ngrams)
    st, ln = TX.ngrams(data, 2)
    emit.spans(st, ln, text=data)


def bigrams(data: bytes):
    """Byte strings of every bigram of ``data`` (the oracle's definition)."""
    for line in data.split(b"\n"):
        toks = [(m.start(), m.end()) for m in _TOKEN.finditer(line)]
        for (s0, _e0), (_s1, e1) in zip(toks, toks[1:]):
            yield line[s0:e1]


def mapfn(key, value, emit):
    with open(value["file"] if isinstance(value, dict) else value, "rb") as f:
        data = f.read()
    for b in bigrams(data):
        emit(b.decode("utf-8", "surrogateescape"), 1)


device_partition = ("fnv1", NUM_REDUCERS)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    emit(sum(values))


combinerfn = reducefn
device_reduce = "sum"
associative_reducer = True
commutative_reducer = True
idempotent_reducer = True


def finalfn(pairs_iterator):
    global RESULT
    out = {}
    for key, values in pairs_iterator:
        out[key] = values[0]
    RESULT = {} if QUIET else out
    return True


def naive(splits: list[bytes]) -> dict:
    """Oracle: bigram -> count over every split."""
    out: dict = {}
    for s in splits:
        for b in bigrams(s):
            k = b.decode("utf-8", "surrogateescape")
            out[k] = out.get(k, 0) + 1
    return out
