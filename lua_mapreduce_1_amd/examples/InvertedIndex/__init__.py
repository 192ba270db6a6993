"""Inverted index as a MapReduce job: word -> sorted distinct line numbers
(BASELINE.json config "inverted-index build on the same corpus shape":
variable-length emit, shuffle skew).  One module holds every function, like
the reference's single-module WordCount (examples/WordCount/init.lua).

* ``taskfn``: one map job per split.  ``init({"nsplits": N, ...})`` for splits
  staged by the SPMD engine (``device_input = "split"``, a SplitStore or
  ``execute_spmd --split-glob``); ``init({"files": [...], ...})`` for
  server/worker or host-plane runs, where each job value carries the file and
  the global number of its first line.
* map: every whitespace token -> (word, global line).  Device form:
  ``emit.word_lines(data)`` (csrc/hip/invidx.hip: tokenizer + LDS vocabulary
  + 64-bit posting keys); host form reads the file.
* partition: exact FNV-1 of the word mod R (examples/WordCount/partitionfn.lua).
* reduce: the sorted distinct line numbers of a word (``device_reduce =
  "concat_unique"``: radix sort + unique of the postings on the device);
  it is also the combiner, and associative/commutative/idempotent.
* finalfn: keeps the index in ``RESULT`` (word -> lines) unless
  ``{"quiet": true}``; returns True.
"""
from __future__ import annotations

NUM_REDUCERS = 10
NSPLITS = 197
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


def _file_lines(path: str) -> int:
    """Lines of a file as the split store numbers them (a file that does not
    end in a newline gets a terminating one)."""
    with open(path, "rb") as f:
        data = f.read()
    return data.count(b"\n") + (0 if data[-1:] == b"\n" else 1)


def taskfn(emit):
    if FILES:
        line0 = 0
        for i, f in enumerate(FILES):
            emit(i + 1, {"file": f, "line0": line0, "split": i})
            line0 += _file_lines(f)
    else:
        for i in range(NSPLITS):
            emit(i + 1, {"split": i})


# the job list is a pure function of the init args: SPMD ranks evaluate it locally
spmd_replicated_taskfn = True
device_input = "split"


def device_mapfn(keys, data, emit):
    emit.word_lines(data)


def mapfn(key, value, emit):
    with open(value["file"], "rb") as f:
        data = f.read()
    if data[-1:] != b"\n":
        data += b"\n"
    for n, line in enumerate(data.split(b"\n")):
        for w in line.split():
            emit(w.decode("utf-8", "surrogateescape"), value["line0"] + n)


device_partition = ("fnv1", NUM_REDUCERS)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    for v in sorted(set(values)):
        emit(v)


combinerfn = reducefn
device_reduce = "concat_unique"
associative_reducer = True
commutative_reducer = True
idempotent_reducer = True


def finalfn(pairs_iterator):
    global RESULT
    out = {}
    n = 0
    for key, values in pairs_iterator:
        n += 1
        if not QUIET:
            out[key] = list(values)
    RESULT = out
    return True


def naive_index(splits: list[bytes]) -> dict:
    """Oracle: word -> sorted distinct global line numbers (split-store layout:
    a split that does not end in a newline is followed by one)."""
    out: dict = {}
    line = 0
    for s in splits:
        if s[-1:] != b"\n":
            s = s + b"\n"
        pieces = s.split(b"\n")
        for n, ln in enumerate(pieces):
            for w in ln.split():
                out.setdefault(w.decode("utf-8", "surrogateescape"), set()).add(line + n)
        line += len(pieces) - 1
    return {k: sorted(v) for k, v in out.items()}
