#!/usr/bin/env python
"""A/B of the record plane's TeraSort kernels on 10 GB (100 M x 100-byte rows
generated in HBM): the row gather (16-byte LDS-staged vs the dword gather)
and the onesweep tile size of the u32-key sort passes, each checked equal to
the default and timed with HIP events (median of --reps).

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
    res["sort_ms"] = timed(lambda: perms.__setitem__(0, RC.sort(rec, TS.KEY, k32, gh)[0]), a.reps)
    from lua_mapreduce_1_amd.ops import _hip
    for r in (24, 40, 48, 32):  # onesweep keys per thread of the u32-key passes (32 = the default, restored last)
        assert _hip.lib().mr_sort_set_rounds32(r) == 0
        res[f"sort_rounds{r}_ms"] = timed(lambda: RC.sort(rec, TS.KEY, k32, gh), a.reps)
        res[f"sort_rounds{r}_equal"] = bool(torch.equal(RC.sort(rec, TS.KEY, k32, gh)[0], perms[0]))
    perm = perms[0]
    outs = {}
    for mode in (0, 1):
        res[f"gather{mode}_ms"] = timed(lambda m=mode: outs.__setitem__(m, RC.gather(rec, perm, mode=m)), a.reps)
    res["gather_modes_equal"] = bool(torch.equal(outs[0], outs[1]))
    outs.clear()
    res["order_ok"] = RC.unsorted_pairs(RC.gather(rec, perm), TS.KEY) == 0
    print(json.dumps(res), flush=True)
    ok = res["gather_modes_equal"] and res["order_ok"] and all(v for k, v in res.items() if k.endswith("_equal"))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
