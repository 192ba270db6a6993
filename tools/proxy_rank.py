#!/usr/bin/env python
"""Per-rank proxy of an N-GPU headline run on ONE GPU: the SPMD word count over
the first 197/N splits (what one rank maps at N GPUs, without the all-to-all),
to measure the fixed per-iteration costs that bound strong scaling.

    python tools/proxy_rank.py --of 8 [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import MODEL, load_corpus  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--of", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--freeze", action="store_true", help="gc.freeze() after warm-up")
    ap.add_argument("--no-prefetch", action="store_true")
    a = ap.parse_args()
    rank, world, device = D.init_from_env()
    splits = load_corpus(1234, 0, 0, 1, device)
    k = (len(splits) + a.of - 1) // a.of
    store = SplitStore(splits[:k])
    params = dict(taskfn=MODEL, mapfn=MODEL, partitionfn=MODEL, reducefn=MODEL, finalfn=MODEL,
                  init_args={"nsplits": k, "num_reducers": 10})
    eng = SPMDEngine(params, device=device, split_store=store)
    eng.prefetch = not a.no_prefetch
    eng.pipeline = os.environ.get("MR_PIPELINE", "1") != "0"
    for w in range(a.warmup):
        eng.run_iteration(prefetch_next=w < a.warmup - 1, lookahead=a.warmup - 1 - w)
    torch.cuda.synchronize()
    if a.freeze:
        import gc
        gc.collect()
        gc.freeze()
    per = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        t1 = time.perf_counter()
        res = eng.run_iteration(prefetch_next=i < a.steps - 1, lookahead=a.steps - 1 - i)
        per.append(1000 * (time.perf_counter() - t1))
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / a.steps
    seq = [round(x, 2) for x in per]
    per.sort()
    print(json.dumps({"of": a.of, "splits": k, "bytes": int(store.offsets[-1]), "ms_per_step": ms, "seq": seq,
                      "min": per[0], "median": per[len(per) // 2], "max": per[-1],
                      "timings": res.timings}), flush=True)
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    if os.environ.get("MR_FAST_EXIT"):
        os._exit(rc)
    sys.exit(rc)
