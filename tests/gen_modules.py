"""User modules of the general-device-plane tests (importable by spawned
ranks).  One module, behaviour picked by ``init({"mode": ...})``, which also
sets ``device_reduce`` (read by the engine after init):

* ``max_host``  — no device_reduce, reducefn = max: the device groups the
  values and the host reducefn folds them (the old silent-``sum`` trap);
* ``docs`` / ``docs_concat`` — int64 values above 2^32 per token,
  ``concat_unique`` / ``concat`` lists;
* ``mixed``     — spans plus host pairs into an ``i64:sum, i64:max`` fold.

Value of a token occurrence: ``len << 40 | next_len << 8 | terminator``,
where next_len is the length of the next token on the same line (0 if none)
and terminator the byte after the token — chunking-invariant, so the oracle
computes it per split.
"""
from __future__ import annotations

import re

import torch

MODE = "max_host"
NSPLITS = 4
FILES: list = []
NUM_REDUCERS = 5
RESULT: dict = {}
device_input = "split"
spmd_replicated_taskfn = True
device_partition = ("fnv1", NUM_REDUCERS)
device_reduce = None
_TOK = re.compile(rb"[^ \t\n\v\f\r]+")


def init(args):
    global MODE, NSPLITS, NUM_REDUCERS, FILES, device_reduce, device_partition
    args = args or {}
    MODE = args.get("mode", MODE)
    FILES = list(args.get("files") or [])
    NSPLITS = int(args.get("nsplits", len(FILES) or NSPLITS))
    NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    device_partition = ("fnv1", NUM_REDUCERS)
    device_reduce = {"max_host": None, "docs": "concat_unique", "docs_concat": "concat",
                     "mixed": ("i64:sum", "max"), "pairs_host": "i64:sum"}[MODE]


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"file": FILES[i], "split": i} if FILES else {"split": i})


def _token_values(data: torch.Tensor):
    from lua_mapreduce_1_amd.ops import text as TX
    st, ln, line = TX.tokens(data, lines=True)
    n = st.numel()
    if n == 0:
        return st, ln, st
    nxt = torch.zeros(n, dtype=torch.int64, device=data.device)
    if n > 1:
        same = line[1:] == line[:-1]
        nxt[:-1] = torch.where(same, ln[1:].to(torch.int64), torch.zeros_like(nxt[:-1]))
    end = st + ln.to(torch.int64)
    term = torch.full((n,), 10, dtype=torch.int64, device=data.device)
    inside = end < data.numel()
    term[inside] = data[end[inside]].to(torch.int64)
    val = (ln.to(torch.int64) << 40) | (nxt << 8) | term
    return st, ln, val


def device_mapfn(key, data, emit):
    if not hasattr(data, "data_ptr"):  # server/worker: the job's file
        from lua_mapreduce_1_amd.ops import io as _io
        data = _io.load_file(data["file"], emit.device)
    if MODE == "pairs_host":
        # a host pair first (the key source becomes a copy of the arena), then
        # pre-encoded keys whose rep words are relative to the mapped chunk
        # (chunk offsets must survive the copy)
        from lua_mapreduce_1_amd import ops
        emit("__host_key__", 1)
        hi, lo, rep = ops.tokenize(data)
        emit.pairs(hi, lo, 1, rep=rep)
        return
    st, ln, val = _token_values(data)
    if MODE == "mixed":
        emit.spans(st, ln, val, val, text=data)
        for _ in range(len(key) if isinstance(key, list) else 1):  # once per job of the chunk
            emit("__host_key__", 5, 5)
            emit("__a_long_host_key_of_many_bytes__", 7, 7)
    else:
        emit.spans(st, ln, val, text=data)


def host_values(split: bytes):
    """(word, value) of every token occurrence of a split (oracle)."""
    out = []
    for line in split.split(b"\n"):
        toks = [(m.start(), m.end()) for m in _TOK.finditer(line)]
        for i, (s, e) in enumerate(toks):
            nxt = toks[i + 1][1] - toks[i + 1][0] if i + 1 < len(toks) else 0
            term = line[e] if e < len(line) else 10
            out.append((line[s:e].decode("utf-8", "surrogateescape"), ((e - s) << 40) | (nxt << 8) | term))
    return out


def mapfn(key, value, emit):
    with open(value["file"], "rb") as f:
        data = f.read()
    for k, v in host_values(data if data.endswith(b"\n") else data + b"\n"):
        emit(k, v)
    if MODE == "mixed":
        emit("__host_key__", 5)
        emit("__a_long_host_key_of_many_bytes__", 7)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    if MODE == "max_host":
        emit(max(values))
    elif MODE == "docs":
        for v in sorted(set(values)):
            emit(v)
    elif MODE == "mixed":
        emit(sum(values))
        emit(max(values))
    else:
        for v in values:
            emit(v)


def finalfn(pairs):
    global RESULT
    RESULT = {k: list(v) for k, v in pairs}
    return True


def oracle(splits: list[bytes], mode: str) -> dict:
    acc: dict = {}
    for s in splits:
        if not s.endswith(b"\n"):
            s = s + b"\n"
        for k, v in host_values(s):
            acc.setdefault(k, []).append(v)
    if mode == "max_host":
        return {k: [max(v)] for k, v in acc.items()}
    if mode == "docs":
        return {k: sorted(set(v)) for k, v in acc.items()}
    if mode == "docs_concat":
        return acc
    out = {k: [sum(v), max(v)] for k, v in acc.items()}
    out["__host_key__"] = [5 * len(splits), 5]
    out["__a_long_host_key_of_many_bytes__"] = [7 * len(splits), 7]
    return out
