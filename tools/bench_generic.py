#!/usr/bin/env python
"""Throughput of the general device plane (parallel/generic.py) on two jobs
that are not word count, through the MapReduce API on mr.spmd:

* bigram: examples/Bigram (byte-span keys = two consecutive tokens of a
  line, int64 sum) over bench.py's Europarl-shaped corpus (197 splits,
  291 MB, ~47 M bigrams);
* scores: examples/ScoreStats (CSV ``word,score``: field split + decimal
  parse on the GPU, typed f64 mean / f64 max / count folds) over a generated
  CSV (``--score-lines`` lines).

Input is staged from pinned host memory every step, like the headline.  The
first warm-up iteration of each job is checked against the module's naive
oracle on a subset of splits (exact equality; float means within 1e-9).
Prints one JSON line per job.

    python tools/bench_generic.py [--steps K] [--warmup W] [--jobs bigram,scores]
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import corpus_dir, ensure_corpus  # noqa: E402
from lua_mapreduce_1_amd import spmd  # noqa: E402
from lua_mapreduce_1_amd.parallel.spmd import SplitStore  # noqa: E402
from lua_mapreduce_1_amd.utils import corpus  # noqa: E402


def _time(eng, steps: int, warmup: int, device) -> float:
    """bench.py's schedule: input copies of the next iteration prefetched and
    its map pipelined (where the plane supports it), but neither the last
    warm-up step nor the last timed step starts work for the one after it."""
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    eng.prefetch, eng.pipeline = True, TUNABLES.pipeline
    for w in range(warmup):
        eng.run_iteration(prefetch_next=w < warmup - 1, lookahead=warmup - 1 - w)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(steps):
        res = eng.run_iteration(prefetch_next=k < steps - 1, lookahead=steps - 1 - k)
    torch.cuda.synchronize(device)
    return (time.perf_counter() - t0) * 1000.0 / steps, res


def _close(a, b) -> bool:
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(_close(x, y) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        return math.isclose(float(a), float(b), rel_tol=1e-9, abs_tol=1e-9)
    return a == b


def _check(mod_name: str, splits: list[bytes], device) -> bool:
    mod = importlib.import_module(mod_name)
    M = mod_name
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                    init_args={"nsplits": len(splits), "num_reducers": 8}), device=device,
               split_store=SplitStore(splits))
    eng.run()
    want = mod.naive(splits)
    got = mod.RESULT
    return got.keys() == want.keys() and all(_close(got[k], want[k]) for k in want)


def run_job(name: str, mod_name: str, store, nbytes: int, check_splits: list[bytes], units: int, unit: str,
            args, device) -> dict:
    M = mod_name
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                    init_args={"nsplits": len(store), "num_reducers": 10, "quiet": True}), device=device,
               split_store=store)
    ms, res = _time(eng, args.steps, args.warmup, device)
    # read the result before the check runs another engine (result columns
    # alias the process's pinned download buffers until the next tail)
    out = {"metric": f"{name} {unit}/s (general device plane, mr.spmd)", "value": units / (ms / 1000.0),
           "unit": f"{unit}/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
           "bytes": int(nbytes), "GB_per_s": nbytes / (ms / 1000.0) / 1e9, "distinct_keys": res.distinct_keys,
           "total_value": res.total_value, "timings_last_step": res.timings}
    del res
    out["oracle_subset_ok"] = _check(mod_name, check_splits, device)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--jobs", default="bigram,scores")
    ap.add_argument("--score-lines", type=int, default=8_000_000)
    args = ap.parse_args()
    device = torch.device("cuda", 0)
    rc = 0
    jobs = args.jobs.split(",")
    if "bigram" in jobs:
        cdir = corpus_dir(1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
        ensure_corpus(cdir, 1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
        off = np.load(os.path.join(cdir, "off.npy"))
        with open(os.path.join(cdir, "blob.bin"), "rb") as f:
            blob = f.read()
        buf = np.frombuffer(blob, np.uint8)
        from lua_mapreduce_1_amd.ops import keys as K
        starts, _ = K.token_spans(buf)
        line = np.searchsorted(np.flatnonzero(buf == 10), starts, side="left")
        per_line = np.bincount(line)
        bigrams = int(np.maximum(per_line - 1, 0).sum())  # consecutive tokens of one line
        sub = [blob[off[i]:off[i + 1]] for i in range(8)]
        del buf, blob
        store = SplitStore.from_blob(os.path.join(cdir, "blob.bin"), off)
        store.finish_loading()
        out = run_job("bigram count", "lua_mapreduce_1_amd.examples.Bigram", store, int(off[-1]), sub, bigrams,
                      "bigrams", args, device)
        out["bigrams_expected"] = bigrams
        out["bigrams_counted"] = out["total_value"]
        rc |= 0 if (out["oracle_subset_ok"] and out["total_value"] == bigrams) else 3
        print(json.dumps(out), flush=True)
    if "scores" in jobs:
        t0 = time.time()
        splits = corpus.score_csv(seed=11, lines=args.score_lines, vocab_size=300_000,
                                  split_lines=max(1, args.score_lines // 197))
        print(f"# generated {args.score_lines} CSV lines in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        out = run_job("CSV group-by mean/max/count", "lua_mapreduce_1_amd.examples.ScoreStats", SplitStore(splits),
                      sum(len(x) for x in splits), splits[:4], args.score_lines, "rows", args, device)
        rc |= 0 if out["oracle_subset_ok"] else 3
        print(json.dumps(out), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
