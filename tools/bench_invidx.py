#!/usr/bin/env python
"""Inverted-index build benchmark (BASELINE.json config "inverted-index build
on the same corpus shape"): the 197-split Europarl-shaped corpus -> word ->
sorted distinct line ids, resident in HBM.  One step = H2D of the rank's
splits + map (tokenize, word ids, posting keys) + sort/unique + (N>1) RCCL
shuffle + merge + key bytes.  Prints one JSON line (tokens/s, postings/s).

  python tools/bench_invidx.py [--steps K] [--warmup W] [--validate]
  (N>1: python -m torch.distributed.run --nproc-per-node N tools/bench_invidx.py)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_corpus  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.invidx import InvertedIndexBuilder, naive_index  # noqa: E402
from lua_mapreduce_1_amd.parallel.spmd import SplitStore  # noqa: E402
from lua_mapreduce_1_amd.utils import corpus  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--reducers", type=int, default=10)
    ap.add_argument("--validate", action="store_true", help="diff 1/8 of the splits against the naive oracle")
    args = ap.parse_args()
    rank, world, device = D.init_from_env()
    splits = load_corpus(args.seed, rank, int(os.environ.get("LOCAL_RANK", 0)), world, device)
    store = SplitStore(splits)
    b = InvertedIndexBuilder(store, device=device, num_reducers=args.reducers)
    # the next build's copies overlap this build's sort (two arenas); neither
    # the last warm-up build nor the last timed one starts anything ahead, so
    # every copy of the timed builds is inside the timed region
    for w in range(args.warmup):
        sh = b.build(prefetch_next=w < args.warmup - 1)
    D.barrier(device=device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        sh = b.build(prefetch_next=i < args.steps - 1)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    D.barrier(device=device)
    ms = 1000.0 * D.all_reduce_max(time.perf_counter() - t0, device) / max(1, args.steps)
    words = D.all_reduce_sum_int(sh.num_words, device)
    postings = D.all_reduce_sum_int(sh.num_postings, device)
    ok = None
    if args.validate and world == 1:
        sub = splits[:len(splits) // 8]
        sb = InvertedIndexBuilder(SplitStore(sub), device=device, num_reducers=args.reducers)
        ok = sb.build().to_host() == naive_index(sub)
    if rank == 0:
        print(f"# phases (last step, s): {b.timings}", file=sys.stderr)
        tokens = corpus.EUROPARL_WORDS
        print(json.dumps({
            "metric": "inverted-index build tokens/s (whole node), Europarl-v7-shaped 197 splits",
            "value": tokens / (ms / 1000.0), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
            "postings_per_s": postings / (ms / 1000.0), "distinct_words": words, "postings": postings,
            "validated_subset": ok, "data": "synthetic Europarl-v7-shaped corpus, host-pinned, staged every step",
            "config": {"model": "inverted index (word -> sorted distinct line ids)", "parallelism": f"dp{world}",
                       "num_reducers": args.reducers}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
