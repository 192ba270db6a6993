"""SPMD test module whose keys overlap in their source: the key of every
whitespace token is the WIDTH-byte window starting at it, cut at the end of
its line (a staged chunk may hold several splits back to back).  Distinct
keys then hold about WIDTH times the split's bytes of key bytes, more than the
single-sync send buffer sized from the row bound holds (the capacity redo of the count exchange must grow the buffer
from the reported totals, not from the bound)."""
import torch

NUM_REDUCERS = 7
NSPLITS = 4
WIDTH = 96


def init(args):
    global NUM_REDUCERS, NSPLITS, device_partition
    if isinstance(args, dict):
        NSPLITS = int(args.get("nsplits", NSPLITS))
        NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    device_partition = ("fnv1", NUM_REDUCERS)


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"split": i})


spmd_replicated_taskfn = True
device_input = "split"
device_partition = ("fnv1", NUM_REDUCERS)


def device_mapfn(key, data, emit):
    from lua_mapreduce_1_amd.ops import text as TX
    st, _ln = TX.tokens(data)
    nl = TX.find_byte(data, 10)
    end = torch.full_like(st, data.numel())
    if nl.numel():
        i = torch.searchsorted(nl, st)
        end = torch.where(i < nl.numel(), nl[i.clamp(max=nl.numel() - 1)], end)
    ln = (end - st).clamp(max=WIDTH).to(torch.int32)
    emit.spans(st, ln, text=data)


def windows(split: bytes):
    import re
    for line in split.split(b"\n"):
        for m in re.finditer(rb"[^ \t\n\v\f\r]+", line):
            yield line[m.start():m.start() + WIDTH]


def mapfn(key, value, emit):
    for w in windows(value):
        emit(w.decode("utf-8", "surrogateescape"), 1)


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
    return True
