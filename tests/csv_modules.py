"""User module of the fused CSV fold tests (``emit.csv``): rows
``f0,f1,...`` with a configurable key field and value fields; mode ``fused``
maps with ``emit.csv`` (one kernel on the GPU), mode ``chain`` with the
ops/text.py chain it is specified by (``TX.csv_rows`` + ``emit.spans``).
Reduce: ("f64:sum", "f64:min", "count") of inputs (VALUES[0], VALUES[1], 1)."""
from __future__ import annotations

import random

MODE = "fused"
NSPLITS = 4
NUM_REDUCERS = 5
KEY = 1
VALUES = (2, 0, None)
SEP = ","
device_input = "split"
spmd_replicated_taskfn = True
device_partition = ("fnv1", NUM_REDUCERS)
device_reduce = ("f64:sum", "f64:min", "count")


def init(args):
    global MODE, NSPLITS, NUM_REDUCERS, KEY, VALUES, SEP, device_partition
    args = args or {}
    MODE = args.get("mode", MODE)
    NSPLITS = int(args.get("nsplits", NSPLITS))
    NUM_REDUCERS = int(args.get("num_reducers", NUM_REDUCERS))
    KEY = int(args.get("key", KEY))
    VALUES = tuple(args.get("values", VALUES))
    SEP = args.get("sep", SEP)
    device_partition = ("fnv1", NUM_REDUCERS)


def taskfn(emit):
    for i in range(NSPLITS):
        emit(i + 1, {"split": i})


def device_mapfn(key, data, emit):
    if MODE == "fused":
        emit.csv(data, key=KEY, values=VALUES, sep=SEP)
    else:
        from lua_mapreduce_1_amd.ops import text as TX
        ks, kl, cols = TX.csv_rows(data, KEY, VALUES, SEP)
        emit.spans(ks, kl, *cols, text=data)


def partitionfn(key):
    h = 2166136261
    for c in key.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ c
    return h % NUM_REDUCERS


def reducefn(key, values, emit):
    raise NotImplementedError("device_reduce only")


GOOD = ["-12", "3.5", " 7 ", "1e3", "+2.25", "0.75", "-0.5", "1024", "2.5E-1"]
BAD = ["abc", "", "1.5x", "-", "e5"]


def make_splits(seed: int = 0, lines: int = 20_000, nsplits: int = 4, long_every: int = 997,
                nkeys: int = 300) -> list[bytes]:
    """Rows with 1..6 fields, empty and long keys, CRLF endings, malformed
    numbers, lines longer than a kernel tile; the last split has no final
    newline."""
    rng = random.Random(seed)
    keys = [f"k{i}" for i in range(nkeys)] + [f"a_rather_long_key_number_{i:04d}" for i in range(40)] + [""]
    out = []
    per = lines // nsplits
    for s in range(nsplits):
        rows = []
        for i in range(per):
            nf = rng.choice([1, 2, 3, 3, 4, 4, 4, 5, 6])
            f = []
            for j in range(nf):
                if j == KEY:
                    f.append(rng.choice(keys))
                elif rng.random() < 0.04:
                    f.append(rng.choice(BAD))
                elif rng.random() < 0.5:
                    f.append(rng.choice(GOOD))
                else:
                    f.append(str(rng.randint(-4000, 4000) * 0.25))
            if long_every and i % long_every == 5:
                f.append("x" * rng.randint(9000, 20000))  # a line across kernel tiles
            rows.append(SEP.join(f) + ("\r" if rng.random() < 0.2 else ""))
        body = "\n".join(rows)
        out.append((body if s == nsplits - 1 else body + "\n").encode())
    return out


def oracle(splits: list[bytes], key: int = None, values=None, sep: str = None) -> dict:
    key = KEY if key is None else key
    values = VALUES if values is None else values
    sep = (SEP if sep is None else sep).encode()
    acc: dict = {}
    for s in splits:
        for line in s.split(b"\n"):
            if line.endswith(b"\r"):
                line = line[:-1]
            f = line.split(sep)
            if len(f) <= key or not f[key]:
                continue
            vals = []
            try:
                for v in values:
                    if v is None:
                        vals.append(1.0)
                    else:
                        if len(f) <= v:
                            raise ValueError
                        vals.append(float(f[v]))
            except ValueError:
                continue
            a = acc.setdefault(f[key].decode("utf-8", "surrogateescape"), [0.0, float("inf"), 0])
            a[0] += vals[0]
            a[1] = min(a[1], vals[1])
            a[2] += 1
    return acc
