"""A host-only word count (plain ``mapfn``, no ``device_mapfn``) over the
synthetic corpus of tests/test_world8.py: runs on the host plane of the SPMD
engine (parallel/spmd_host.py).  Keys mix strings and tuples (a (word, length)
key for every word of 6+ bytes), values are ints and tuples, so the shuffle
carries the reference's tuple-wrapped keys and values (job.lua:83-97)."""
from __future__ import annotations

NSPLITS = 16
NUM_REDUCERS = 10
SEED = 21
_SPLITS: list = []
RESULT: dict = {}


def init(args):
    global NSPLITS, NUM_REDUCERS, SEED, _SPLITS
    args = args or {}
    NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    SEED = int(args.get("seed", SEED))
    _SPLITS = corpus(SEED, int(args.get("lines", 4000)))
    NSPLITS = len(_SPLITS)


def corpus(seed: int, lines: int) -> list:
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    return europarl_like(seed=seed, lines=lines, words=15 * lines, vocab_size=4000, split_lines=250)


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, i)


def mapfn(key, value, emit):
    for w in _SPLITS[value].split():
        s = w.decode("utf-8", "surrogateescape")
        emit(s, 1)
        if len(w) >= 6:
            emit((s[:3], len(w)), (1, len(w)))


def partitionfn(key):
    s = key if isinstance(key, str) else "%s/%d" % key
    h = 2166136261
    for c in s.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    if isinstance(key, str):
        emit(sum(values))
    else:
        emit((sum(v[0] for v in values), sum(v[1] for v in values)))


def finalfn(pairs):
    global RESULT
    RESULT = {k: list(v) for k, v in pairs}
    return True


def naive(splits) -> dict:
    acc: dict = {}
    for s in splits:
        for w in s.split():
            k = w.decode("utf-8", "surrogateescape")
            acc[k] = acc.get(k, 0) + 1
            if len(w) >= 6:
                t = (k[:3], len(w))
                a = acc.get(t, (0, 0))
                acc[t] = (a[0] + 1, a[1] + len(w))
    return {k: [v] for k, v in acc.items()}
