#!/usr/bin/env python
"""A/B of the record plane's TeraSort kernels on 10 GB (100 M x 100-byte rows
generated in HBM): the row gather (16-byte LDS-staged vs the dword gather)
and the tie fix-up (scan + per-run fix vs the single kernel), each checked
equal to the other and timed with HIP events (median of --reps).

    python tools/ts_ab.py [--rows 100000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import records as RC  # noqa: E402
from lua_mapreduce_1_amd.ops import terasort as TS  # noqa: E402


def timed(fn, reps: int) -> float:
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return statistics.median(out)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    rec = TS.generate(a.rows, 0, 42, d)
    torch.cuda.synchronize()
    gh = torch.zeros(2048, dtype=torch.int32, device=d)
    k32 = RC.keys32(rec, TS.KEY, gh)
    res = {"rows": a.rows}
    res["keys32_ms"] = timed(lambda: RC.keys32(rec, TS.KEY, torch.zeros(2048, dtype=torch.int32, device=d)), a.reps)
    perms = {}
    for mode in (0, 1):
        res[f"sort_tie{mode}_ms"] = timed(lambda m=mode: perms.__setitem__(m, RC.sort(rec, TS.KEY, k32, gh,
                                                                                       tie_mode=m)[0]), a.reps)
    res["tie_modes_equal"] = bool(torch.equal(perms[0], perms[1]))
    perm = perms[0]
    outs = {}
    for mode in (0, 1):
        res[f"gather{mode}_ms"] = timed(lambda m=mode: outs.__setitem__(m, RC.gather(rec, perm, mode=m)), a.reps)
    res["gather_modes_equal"] = bool(torch.equal(outs[0], outs[1]))
    outs.clear()
    res["order_ok"] = RC.unsorted_pairs(RC.gather(rec, perm), TS.KEY) == 0
    print(json.dumps(res), flush=True)
    ok = res["tie_modes_equal"] and res["gather_modes_equal"] and res["order_ok"]
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
