"""Record-plane test module: random fixed-width rows of any shape
(``init({"rb": row bytes, "kb": key bytes, "rows": n, "blocks": B,
"partitions": R, "skew": bool})``), an identity map through
``emit.records(rec, kb)``; finalfn keeps every row in result-file order.
With ``skew`` most keys share a 4-byte prefix (runs longer than the tie
fix-up handles: the full-key fallback sort)."""
import numpy as np
import torch

RB, KB, ROWS, BLOCKS, PARTITIONS, SKEW = 64, 16, 10000, 3, 4, False
RESULT: list = []
spmd_replicated_taskfn = True
device_reduce = "identity"
device_partition = ("range", PARTITIONS, None)


def init(args):
    global RB, KB, ROWS, BLOCKS, PARTITIONS, SKEW, device_partition
    RB, KB = int(args.get("rb", RB)), int(args.get("kb", KB))
    ROWS, BLOCKS = int(args.get("rows", ROWS)), int(args.get("blocks", BLOCKS))
    PARTITIONS, SKEW = int(args.get("partitions", PARTITIONS)), bool(args.get("skew", False))
    device_partition = ("range", PARTITIONS, None)


def block_rows(b: int) -> np.ndarray:
    per = ROWS // BLOCKS
    n = per if b < BLOCKS - 1 else ROWS - per * (BLOCKS - 1)
    rng = np.random.default_rng(1000 + b)
    a = rng.integers(0, 256, (n, RB), dtype=np.uint8)
    if SKEW:
        a[: n * 3 // 4, : min(4, KB)] = 7  # a shared prefix: runs of thousands of equal 32-bit prefixes
        a[: n // 2, : KB] = a[0, : KB]     # and exact duplicate keys
    return a


def taskfn(emit):
    for b in range(BLOCKS):
        emit(b + 1, {"block": b})


def device_mapfn(key, value, emit):
    emit.records(torch.from_numpy(block_rows(value["block"])).to(emit.device), KB)


def partitionfn(key):
    return 0


def reducefn(key, values, emit):
    for v in values:
        emit(v)


def finalfn(pairs):
    global RESULT
    RESULT = [(k, v[0]) for k, v in pairs]
    return True
