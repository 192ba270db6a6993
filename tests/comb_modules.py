"""User modules of the combiner / batched-reducer tests (importable by
spawned ranks).  Behaviour picked by ``init({"mode": ...})``:

* ``host``   — WordCount with reducefn2's contract: sum reducer, combinerfn =
  reducefn, no ACI flags, no device hooks (host combiner per key);
* ``device`` — the same with ``device_reducefn`` (segments.sum): batched
  combiner and reducer on the device;
* ``topk``   — per token the 3 largest token values (gen_modules values),
  variable-length ValueLists from the device, combinerfn = reducefn;
* ``median`` — per token [median, distinct count] of its values, NO combiner
  (a median does not combine), device_reducefn returns two columns;
* ``hot``    — word count plus one hot key with HOT values per split.
"""
from __future__ import annotations

import statistics

import torch

from gen_modules import _token_values, host_values  # noqa: F401  (same token values)

MODE = "host"
NSPLITS = 4
NUM_REDUCERS = 5
HOT = 0
RESULT: dict = {}
CALLS = {"combinerfn": 0, "reducefn": 0}
device_input = "split"
spmd_replicated_taskfn = True
device_partition = ("fnv1", NUM_REDUCERS)
device_reduce = None
device_reducefn = None
combinerfn = None


def init(args):
    global MODE, NSPLITS, NUM_REDUCERS, HOT, device_partition, device_reducefn, combinerfn
    args = args or {}
    MODE = args.get("mode", MODE)
    NSPLITS = int(args.get("nsplits", NSPLITS))
    NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    HOT = int(args.get("hot", 0))
    device_partition = ("fnv1", NUM_REDUCERS)
    device_reducefn = {"host": None, "device": _dev_sum, "topk": _dev_topk, "median": _dev_median,
                       "hot": _dev_sum if args.get("hot_device") else None}[MODE]
    combinerfn = None if MODE == "median" else reducefn


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"split": i})


def device_mapfn(key, data, emit):
    if MODE in ("topk", "median"):
        st, ln, val = _token_values(data)
        emit.spans(st, ln, val, text=data)
        return
    emit.words(data)
    if MODE == "hot" and HOT:
        hot = torch.frombuffer(bytearray(b"__hot__"), dtype=torch.uint8).to(data.device)
        for _ in range(len(key) if isinstance(key, list) else 1):  # once per split of the chunk
            emit.spans(torch.zeros(HOT, dtype=torch.int64, device=data.device),
                       torch.full((HOT,), 7, dtype=torch.int32, device=data.device), 1, text=hot)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    CALLS["reducefn"] += 1
    if MODE == "topk":
        for v in sorted(values, reverse=True)[:3]:
            emit(v)
    elif MODE == "median":
        emit(float(statistics.median(values)))
        emit(len(set(values)))
    else:
        emit(sum(values))


def _dev_sum(keys, off, val):
    from lua_mapreduce_1_amd.ops import segments as S
    return S.sum(off, val)


def _dev_topk(keys, off, val):
    from lua_mapreduce_1_amd.ops import segments as S
    from lua_mapreduce_1_amd.parallel.reducers import ValueLists
    return ValueLists(*S.topk(off, val, 3))


def _dev_median(keys, off, val):
    from lua_mapreduce_1_amd.ops import segments as S
    return S.median(off, val), S.nunique(off, val)


def finalfn(pairs):
    global RESULT
    RESULT = {k: list(v) for k, v in pairs}
    return True


def oracle(splits: list[bytes], mode: str, hot: int = 0) -> dict:
    acc: dict = {}
    for s in splits:
        if not s.endswith(b"\n"):
            s = s + b"\n"
        if mode in ("topk", "median"):
            for k, v in host_values(s):
                acc.setdefault(k, []).append(v)
        else:
            for w in s.split():
                k = w.decode("utf-8", "surrogateescape")
                acc[k] = acc.get(k, 0) + 1
    if mode == "topk":
        return {k: sorted(v, reverse=True)[:3] for k, v in acc.items()}
    if mode == "median":
        return {k: [float(statistics.median(v)), len(set(v))] for k, v in acc.items()}
    out = {k: [v] for k, v in acc.items()}
    if hot:
        out["__hot__"] = [hot * len(splits)]
    return out
