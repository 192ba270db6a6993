"""Word -> the distinct sources that use it: a MapReduce job with
byte-string values.

Input lines are ``<source>\\t<text>`` (a URL, a file or speaker name, ...).
The reference's values are arbitrary Lua strings, serialised into its
intermediate files (/root/reference/mapreduce/job.lua:84,212-214,
utils.lua:100-120).  Here the map module declares ``device_value_dtype =
"bytes"``: a value is a span of the staged text (the line's source name),
stored as a span word and shuffled with its bytes (parallel/values.py); the
reduce ``concat_unique`` sorts each word's sources by their bytes on the
device and drops duplicates.

* ``taskfn``: one map job per split (``device_input = "split"``);
* map: every token of a line's text -> (token, the line's source); device
  form: newline / tab positions and ``ops/text.py`` tokens, the value column
  ``emit.bytes(starts, lens)``;
* partition: exact FNV-1 of the word mod R;
* reduce: sorted distinct source names (also the combiner).
"""
from __future__ import annotations

import numpy as np
import torch

NUM_REDUCERS = 10
NSPLITS = 8
SPLITS: list = []
FILES: list = []    # server/worker (and host-plane) form: one map job per file
RESULT: dict = {}
device_input = "split"
spmd_replicated_taskfn = True
device_value_dtype = "bytes"
device_reduce = "concat_unique"
device_partition = ("fnv1", NUM_REDUCERS)


def init(args):
    global NUM_REDUCERS, NSPLITS, SPLITS, FILES, device_partition
    args = args or {}
    NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    SPLITS = list(args.get("splits") or [])
    FILES = list(args.get("files") or [])
    NSPLITS = int(args.get("nsplits", len(FILES) or len(SPLITS) or NSPLITS))
    device_partition = ("fnv1", NUM_REDUCERS)


def _file_lines(path: str) -> int:
    with open(path, "rb") as f:
        data = f.read()
    return data.count(b"\n") + (0 if data[-1:] == b"\n" else 1)


def taskfn(emit):
    line0 = 0
    for i in range(NSPLITS):
        if FILES:
            emit(i + 1, {"split": i, "file": FILES[i], "line0": line0})
            line0 += _file_lines(FILES[i])
        else:
            emit(i + 1, {"split": i})


def _data(value, emit):
    if hasattr(value, "data_ptr"):
        return value  # SPMD: the staged split(s)
    from lua_mapreduce_1_amd.ops import io as _io
    return _io.load_file(value["file"], emit.device)  # a worker's job: its file


def _text(value) -> bytes:
    if isinstance(value, dict) and value.get("file"):
        with open(value["file"], "rb") as f:
            return f.read()
    return SPLITS[value["split"]]


def line_sources(data: torch.Tensor):
    """(starts, lens) of every line's source name — the bytes before its
    first tab (empty when the line has none) — and the end of that name per
    line (tokens before it belong to the name)."""
    d = data.device
    nl = torch.nonzero(data == 10).flatten()
    starts = torch.cat([torch.zeros(1, dtype=torch.int64, device=d), nl + 1])
    ends = torch.cat([nl, torch.tensor([data.numel()], dtype=torch.int64, device=d)])
    tabs = torch.nonzero(data == 9).flatten()
    if tabs.numel():
        k = torch.searchsorted(tabs, starts)  # the first tab at or after each line start
        tab = torch.where(k < tabs.numel(), tabs[k.clamp(max=tabs.numel() - 1)], ends)
    else:
        tab = ends
    has = tab < ends
    lens = torch.where(has, tab - starts, torch.zeros_like(tab))
    name_end = torch.where(has, tab, starts - 1)
    return starts, lens, name_end


def device_mapfn(keys, value, emit):
    from lua_mapreduce_1_amd.ops import text as TX
    data = _data(value, emit)
    st, ln, line = TX.tokens(data, lines=True)
    s0, sl, name_end = line_sources(data)
    keep = st > name_end[line]  # the text after the tab (the name itself is no word of it)
    st, ln, line = st[keep], ln[keep], line[keep]
    emit.spans(st, ln, emit.bytes(s0[line], sl[line], text=data), text=data)


def mapfn(key, value, emit):
    s = _text(value)
    for text in s.split(b"\n"):
        name, tab, rest = text.partition(b"\t")
        if not tab:
            name, rest = b"", name
        src = name.decode("utf-8", "surrogateescape")
        for w in rest.split():
            emit(w.decode("utf-8", "surrogateescape"), src)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    for v in sorted(set(values), key=lambda x: x.encode("utf-8", "surrogateescape")):
        emit(v)


combinerfn = reducefn
associative_reducer = True
commutative_reducer = True
idempotent_reducer = True


def finalfn(pairs):
    global RESULT
    RESULT = {k: list(vs) for k, vs in pairs}
    return True


def corpus(seed: int = 3, lines: int = 6000, sources: int = 40, vocab: int = 3000, split_lines: int = 500) -> list:
    """Synthetic ``<source>\\t<text>`` lines: source names of 3-60 bytes
    (some longer than 16, some sharing long prefixes), Zipf-distributed words;
    a few lines without a tab."""
    rng = np.random.default_rng(seed)
    names = []
    for i in range(sources):
        if i % 5 == 0:
            names.append("https://example.org/a/very/long/shared/prefix/%d" % i)
        else:
            names.append("src%d" % i * (1 + i % 3))
    words = ["w%d" % i for i in range(vocab)]
    out, cur = [], []
    for n in range(lines):
        ws = " ".join(words[min(int(x), vocab) - 1] for x in rng.zipf(1.3, 1 + int(rng.integers(0, 12))))
        if n % 97 == 13:
            cur.append(ws)
        else:
            cur.append(names[int(rng.integers(0, sources))] + "\t" + ws)
        if len(cur) == split_lines:
            out.append(("\n".join(cur) + "\n").encode())
            cur = []
    if cur:
        out.append(("\n".join(cur) + "\n").encode())
    return out


def naive(splits: list[bytes]) -> dict:
    out: dict = {}
    for s in splits:
        for text in s.split(b"\n"):
            name, tab, rest = text.partition(b"\t")
            if not tab:
                name, rest = b"", name
            for w in rest.split():
                out.setdefault(w.decode("utf-8", "surrogateescape"), set()).add(name)
    return {k: [v.decode("utf-8", "surrogateescape") for v in sorted(vs)] for k, vs in out.items()}
