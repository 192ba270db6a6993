#!/usr/bin/env python
"""TeraSort-style benchmark (BASELINE.json config "TeraSort-style 10 GB
key/value sort on 8xMI355X (radix sort + all-to-all)").

Records (100 B: 10 B key + 90 B value) are generated in HBM by the TeraGen
analogue kernel (untimed); one timed step = splitter sampling + partition +
all-to-all of the rows (N>1) + local 80-bit radix sort + row gather, output
resident in HBM.  Validation (global order + record checksum) after timing.

  python tools/bench_terasort.py [--gb 10] [--steps K] [--warmup W]
  (N>1: python -m torch.distributed.run --nproc-per-node N tools/bench_terasort.py)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.terasort import TeraSort  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10.0, help="total data size (1 GB = 1e9 bytes)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    rank, world, device = D.init_from_env()
    total = int(args.gb * 1e9) // 100
    t = TeraSort(total, device=device)
    rec = t.generate()
    cs = t.checksum_global(rec)
    out = None
    for _ in range(args.warmup):
        out = t.sort(rec)
        del out
    D.barrier(device=device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = t.sort(rec)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    D.barrier(device=device)
    ms = 1000.0 * D.all_reduce_max(time.perf_counter() - t0, device) / max(1, args.steps)
    v = t.validate(out, cs)
    if rank == 0:
        print(f"# phases (last step, s): {t.timings}; validation {v}", file=sys.stderr)
        gbps = total * 100 / 1e9 / (ms / 1000.0)
        print(json.dumps({
            "metric": "TeraSort-style sort GB/s (whole node), 100-byte records",
            "value": gbps, "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "strong", "records": total,
            "valid": bool(v.get("ok")), "data": "synthetic TeraGen-style records generated in HBM (untimed)",
            "config": {"model": "terasort (10-byte key, 90-byte value)", "total_gb": args.gb,
                       "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
