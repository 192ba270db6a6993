"""Word-count job over host-resident input splits — the benchmark workload.

The reference's headline run (README.md:43-75, examples/WordCountBig/taskfn.lua)
counts the whitespace tokens of Europarl-v7 EN split in 197 files with one map
job per file, the sum reducer as combiner and 10 reduce partitions
(README.md:59).  Here the splits live in a :class:`parallel.spmd.SplitStore`
(pinned host memory standing in for the page cache); ``init(args)`` takes
``{"nsplits": N, "num_reducers": R}``.
"""
NUM_REDUCERS = 10
NSPLITS = 197


def init(args):
    global NUM_REDUCERS, NSPLITS, device_partition
    if isinstance(args, dict):
        NSPLITS = int(args.get("nsplits", NSPLITS))
        NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    device_partition = ("fnv1", NUM_REDUCERS)


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"split": i})


# the job list is a pure function of init args: SPMD ranks evaluate it locally
spmd_replicated_taskfn = True


device_input = "split"


def device_mapfn(keys, data, emit):
    emit.words(data)


def mapfn(key, value, emit):  # host form (value: bytes of the split)
    for w in value.split():
        emit(w.decode("utf-8", "surrogateescape"), 1)


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
    n = 0
    for _key, values in pairs_iterator:
        n += values[0]
    global LAST_TOTAL
    LAST_TOTAL = n
    return True


LAST_TOTAL = 0
