#!/usr/bin/env python
"""TeraSort benchmark (BASELINE.json config "TeraSort-style 10 GB key/value
sort on 8xMI355X (radix sort + all-to-all)") through the MapReduce API: the
examples/TeraSort module (identity map, sampled range partitioner, identity
reduce) on the SPMD engine's record plane.

Each rank's input block (100-byte records) is generated in HBM by the TeraGen
kernel before timing and handed to the engine as a RecordStore; one timed step
= one iteration: map (emit the block) + splitter sampling + partition +
all-to-all of the rows (N>1) + local 80-bit radix sort + row gather, output
resident in HBM.  Validation (global order + record checksum, collective
device_finalfn) after timing.

  python tools/bench_terasort.py [--gb 10] [--steps K] [--warmup W]
  (N>1: python -m torch.distributed.run --nproc-per-node N tools/bench_terasort.py)
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lua_mapreduce_1_amd import spmd  # noqa: E402
from lua_mapreduce_1_amd.ops import terasort as TS  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.planes import RecordStore  # noqa: E402

M = "lua_mapreduce_1_amd.examples.TeraSort"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10.0, help="total data size (1 GB = 1e9 bytes)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2, help="untimed iterations (two: the double-buffered 10 GB outputs are both allocated before timing)")
    args = ap.parse_args()
    rank, world, device = D.init_from_env()
    total = int(args.gb * 1e9) // 100
    mod = importlib.import_module(M)
    mod.init({"records": total, "blocks": world})
    blocks = mod.blocks()
    # every rank generates (only) its own block: block r is rank r's job
    store = RecordStore([TS.generate(n, first, mod.SEED, device) if b == rank else torch.empty(0)
                         for b, (first, n) in enumerate(blocks)])
    for b, (first, n) in enumerate(blocks):
        if b != rank:
            store.blocks[b] = torch.empty((n, TS.REC), dtype=torch.uint8, device="meta")
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"records": total, "blocks": world, "partitions": world})
    eng = spmd(params, device=device, split_store=store)
    for _ in range(args.warmup):
        res = eng.run_iteration()
        del res
    D.barrier(device=device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = eng.run_iteration()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    D.barrier(device=device)
    ms = 1000.0 * D.all_reduce_max(time.perf_counter() - t0, device) / max(1, args.steps)
    timings = res.timings
    del res
    # validation iteration (not timed): input checksum in the map, collective check
    mod.VALIDATE = True
    mod._INPUT_CHECKSUM[0] = 0
    res = eng.run_iteration()
    ok = mod.device_finalfn(res, eng)
    if rank == 0:
        print(f"# phases (last timed step, s): {timings}; validation {mod.VALIDATION}", file=sys.stderr)
        gbps = total * 100 / 1e9 / (ms / 1000.0)
        print(json.dumps({
            "metric": "TeraSort-style sort GB/s (whole node), 100-byte records",
            "value": gbps, "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "strong", "records": total,
            "valid": bool(ok), "data": "synthetic TeraGen-style records generated in HBM (untimed)",
            "config": {"model": "examples/TeraSort (10-byte key, 90-byte value) on mr.spmd", "total_gb": args.gb,
                       "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
