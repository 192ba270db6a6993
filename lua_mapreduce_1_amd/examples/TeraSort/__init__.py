"""TeraSort as a MapReduce job (BASELINE.json config "TeraSort-style 10 GB
key/value sort on 8xMI355X (radix sort + all-to-all)"): 100-byte records with
10-byte keys, identity map, sampled range partitioner, identity reduce — the
framework's shuffle and per-partition key sort do all the work (the
reference's partition / sort / merge path: job.lua:194-215, utils.lua:206-271).

* ``taskfn``: one map job per input block ``{"block": b, "first": r0, "n": n}``
  (``init({"records": N, "blocks": B, "seed": S, "partitions": R})``).
* map: the block's records — a RecordStore block staged by the caller
  (``device_input = "records"``), or generated on the spot by the TeraGen
  analogue (csrc/hip/terasort.hip) — emitted with ``emit.records``.
* partition: ``("range", R, None)``: R-1 splitters sampled from every rank's
  keys (R = 0: one partition per rank).
* reduce: identity (``device_reduce = "identity"``): records sorted by key
  within their partition (radix sort of the 64-bit key prefix + tie fix-up).
* ``device_finalfn`` (SPMD, every rank): order within and across ranks and an
  order-independent record checksum against the input's, when
  ``{"validate": true}``; result in ``VALIDATION``.
* host forms (server/worker): TeraGen on the CPU, uniform static splitters.
"""
from __future__ import annotations

RECORDS = 100_000
BLOCKS = 1
SEED = 0x7E5A
PARTITIONS = 0
VALIDATE = False
VALIDATION: dict = {}
_INPUT_CHECKSUM = [0]


def init(args):
    global RECORDS, BLOCKS, SEED, PARTITIONS, VALIDATE, device_partition
    if isinstance(args, dict):
        RECORDS = int(args.get("records", RECORDS))
        BLOCKS = int(args.get("blocks", BLOCKS))
        SEED = int(args.get("seed", SEED))
        PARTITIONS = int(args.get("partitions", PARTITIONS))
        VALIDATE = bool(args.get("validate", False))
    device_partition = ("range", PARTITIONS, None)
    _INPUT_CHECKSUM[0] = 0


def blocks():
    per = RECORDS // BLOCKS
    return [(b * per, per if b < BLOCKS - 1 else RECORDS - per * (BLOCKS - 1)) for b in range(BLOCKS)]


def taskfn(emit):
    for b, (first, n) in enumerate(blocks()):
        emit(b + 1, {"block": b, "first": first, "n": n})


spmd_replicated_taskfn = True
device_input = "records"


def device_mapfn(key, value, emit):
    from lua_mapreduce_1_amd.ops import terasort as TS
    rec = value if hasattr(value, "data_ptr") else TS.generate(value["n"], value["first"], SEED, emit.device)
    if VALIDATE:
        _INPUT_CHECKSUM[0] = (_INPUT_CHECKSUM[0] + TS.checksum(rec)) & ((1 << 64) - 1)
    emit.records(rec)


def mapfn(key, value, emit):
    from lua_mapreduce_1_amd.ops import terasort as TS
    rec = TS.generate(value["n"], value["first"], SEED).numpy()
    for row in rec:
        b = row.tobytes()
        emit(b[:TS.KEY], b[TS.KEY:])


device_partition = ("range", PARTITIONS, None)


def partitionfn(key):
    # host form: TeraGen keys are uniform -> R equal ranges of the 64-bit prefix
    r = PARTITIONS or 1
    return (int.from_bytes(bytes(key[:8]).ljust(8, b"\0"), "big") * r) >> 64


def reducefn(key, values, emit):
    for v in values:
        emit(v)


device_reduce = "identity"


def device_finalfn(res, eng):
    """Collective check of this iteration's sorted output (every rank)."""
    global VALIDATION
    if not VALIDATE:
        return True
    import torch
    from lua_mapreduce_1_amd.ops import terasort as TS
    from lua_mapreduce_1_amd.parallel import dist as D
    out = res.device["records"]
    hi, lo = TS.keys(out)
    bad = TS.unsorted_pairs(hi, lo)
    n = int(out.shape[0])
    edge = [int(hi[0]), int(lo[0]), int(hi[-1]), int(lo[-1])] if n else None
    m64 = (1 << 64) - 1
    info = D.gather_objects((n, edge, TS.checksum(out), _INPUT_CHECKSUM[0], bad), 0, eng.group)
    ok = True
    if eng.rank == 0:
        u = lambda x: x & m64  # noqa: E731
        cross, prev = 0, None
        for m, e, _c, _i, _b in info:
            if not m:
                continue
            first, last = (u(e[0]), u(e[1])), (u(e[2]), u(e[3]))
            if prev is not None and first < prev:
                cross += 1
            prev = last
        out_cs = sum(x[2] for x in info) & m64
        in_cs = sum(x[3] for x in info) & m64
        VALIDATION = {"records": sum(x[0] for x in info), "unsorted_pairs": sum(x[4] for x in info),
                      "rank_boundary_violations": cross, "checksum_ok": out_cs == in_cs}
        ok = (VALIDATION["records"] == RECORDS and VALIDATION["unsorted_pairs"] == 0 and cross == 0
              and VALIDATION["checksum_ok"])
        VALIDATION["ok"] = ok
    del torch
    return ok


def finalfn(pairs_iterator):
    global VALIDATION
    prev, n, ok = None, 0, True
    for key, _values in pairs_iterator:
        k = key.encode("utf-8", "surrogateescape") if isinstance(key, str) else bytes(key)
        ok &= prev is None or prev <= k
        prev, n = k, n + 1
    VALIDATION = {"records": n, "ok": ok and n == RECORDS}
    return True
