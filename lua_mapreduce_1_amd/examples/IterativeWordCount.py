"""Iterative word count for the SPMD engine: the benchmark job's map/partition/
reduce (models/wordcount.py) with a finalfn that loops ``iterations`` times,
keeping its state in a JSON file (``state_file`` init arg) so it survives a
relaunch — the role the persistent_table plays in the APRIL-ANN example
(examples/APRIL-ANN/common.lua:57-77, 144-202).  Used by the SPMD
checkpoint/resume test: every iteration appends its total token count.
"""
import json
import os

from lua_mapreduce_1_amd.models import wordcount as _wc

STATE_FILE = None
ITERATIONS = 3


def init(args):
    global STATE_FILE, ITERATIONS
    _wc.init(args)
    STATE_FILE = args.get("state_file")
    ITERATIONS = int(args.get("iterations", ITERATIONS))


taskfn = _wc.taskfn
spmd_replicated_taskfn = True
device_input = _wc.device_input
device_mapfn = _wc.device_mapfn
mapfn = _wc.mapfn
partitionfn = _wc.partitionfn
reducefn = _wc.reducefn
device_reduce = _wc.device_reduce
associative_reducer = commutative_reducer = idempotent_reducer = True


def __getattr__(name):  # device_partition follows wordcount.init's num_reducers
    if name == "device_partition":
        return _wc.device_partition
    raise AttributeError(name)


def _load():
    if STATE_FILE and os.path.exists(STATE_FILE):
        with open(STATE_FILE) as f:
            return json.load(f)
    return {"totals": []}


def finalfn(pairs_iterator):
    n = sum(values[0] for _key, values in pairs_iterator)
    st = _load()
    st["totals"].append(n)
    if STATE_FILE:
        tmp = STATE_FILE + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, STATE_FILE)
    return "loop" if len(st["totals"]) < ITERATIONS else True
