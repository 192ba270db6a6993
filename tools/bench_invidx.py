#!/usr/bin/env python
"""Inverted-index benchmark (BASELINE.json config "inverted-index build on the
same corpus shape") through the MapReduce API: the examples/InvertedIndex
module (taskfn / device_mapfn / FNV partitionfn / concat_unique reducefn) on
the SPMD engine's list plane.  Corpus = bench.py's Europarl-shaped 197 splits
(each rank reads and pins only its own).  One step = one iteration: H2D of the
rank's splits + map (tokenizer, vocabulary, posting keys) + sort/unique +
(N>1) RCCL shuffle + merge + (partition, key) order + key bytes; the index
stays in HBM.  Prints one JSON line (tokens/s, postings/s).

  python tools/bench_invidx.py [--steps K] [--warmup W] [--validate]
  (N>1: python -m torch.distributed.run --nproc-per-node N tools/bench_invidx.py)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import corpus_dir, ensure_corpus  # noqa: E402
from lua_mapreduce_1_amd import spmd  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.spmd import SplitStore  # noqa: E402
from lua_mapreduce_1_amd.utils import corpus  # noqa: E402

M = "lua_mapreduce_1_amd.examples.InvertedIndex"


def host_index_digest(blob: bytes) -> dict:
    """word -> (distinct lines, sum of line ids) of the whole corpus, from its
    bytes alone (numpy; independent of the device kernels): tokens are maximal
    runs outside Lua's %s, lines are counted by newlines, words grouped by
    their bytes (the exact 128-bit packing of ops/keys.py for words of <= 15
    bytes, the bytes themselves for longer ones)."""
    from lua_mapreduce_1_amd.ops import keys as K
    buf = np.frombuffer(blob, np.uint8)
    starts, lens = K.token_spans(buf)
    line = np.searchsorted(np.flatnonzero(buf == 10), starts, side="left").astype(np.int64)
    short = lens <= K.PACK_MAX
    hi, lo = K.span_keys(buf, np.where(short, starts, 0), np.where(short, lens, 1))
    out: dict = {}
    # short words: unique (hi, lo, line) triples, then per (hi, lo) count and sum
    rec = np.empty(int(short.sum()), dtype=[("h", "<u8"), ("l", "<u8"), ("n", "<i8")])
    rec["h"], rec["l"], rec["n"] = hi[short], lo[short], line[short]
    rec = np.unique(rec)
    kk = rec[["h", "l"]]
    head = np.ones(rec.size, bool)
    head[1:] = (rec["h"][1:] != rec["h"][:-1]) | (rec["l"][1:] != rec["l"][:-1])
    idx = np.flatnonzero(head)
    cnt = np.diff(np.append(idx, rec.size))
    sums = np.add.reduceat(rec["n"], idx) if rec.size else np.zeros(0, np.int64)
    for i, c, sm in zip(idx.tolist(), cnt.tolist(), sums.tolist()):
        w = K.unpack_key(int(kk[i]["h"]), int(kk[i]["l"]))
        out[w] = (c, sm)
    long_sets: dict = {}
    for s_, n_, l_ in zip(starts[~short].tolist(), lens[~short].tolist(), line[~short].tolist()):
        long_sets.setdefault(blob[s_:s_ + n_], set()).add(l_)
    for w, st in long_sets.items():
        out[w] = (len(st), sum(st))
    return out


def validate_full(eng, res, cdir: str, off, world: int, rank: int) -> bool | None:
    """Every word of the index (all ranks' partitions, gathered on rank 0)
    against host_index_digest of the corpus: same words, same number of
    distinct lines and line-id sum for each."""
    got: dict = {}
    for _name, cols in eng.gather_results(res):
        kb, ko = cols["key_blob"].tobytes(), cols["key_off"]
        lo_, lv = cols["list_off"], cols["list_val"]
        for i in range(int(ko.size) - 1):
            v = lv[lo_[i]:lo_[i + 1]]
            got[kb[ko[i]:ko[i + 1]]] = (int(v.size), int(v.astype(np.int64).sum()))
    if rank != 0:
        return None
    with open(os.path.join(cdir, "blob.bin"), "rb") as f:
        blob = f.read()
    want = host_index_digest(blob)
    return got == want


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--reducers", type=int, default=10)
    ap.add_argument("--validate", action="store_true",
                    help="check the WHOLE index against a host oracle built from the corpus bytes: every word's "
                         "number of distinct lines and the sum of its line ids (plus a 1/8-corpus exact diff)")
    ap.add_argument("--vocab-log2", type=int, default=0, help="vocabulary table capacity 2^k (0 = the plane's default)")
    args = ap.parse_args()
    rank, world, device = D.init_from_env()
    cdir = corpus_dir(args.seed, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
    if int(os.environ.get("LOCAL_RANK", 0)) == 0:
        ensure_corpus(cdir, args.seed, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
    D.barrier(device=device)
    off = np.load(os.path.join(cdir, "off.npy"))
    store = SplitStore.from_blob(os.path.join(cdir, "blob.bin"), off, rank, world, pin=device.type == "cuda")
    store.finish_loading()
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"nsplits": len(store), "num_reducers": args.reducers, "quiet": True})
    if args.vocab_log2:
        params["table_capacity"] = 1 << args.vocab_log2
    eng = spmd(params, device=device, split_store=store)
    # the next iteration's copies overlap this iteration's sort (three
    # arenas); neither the last warm-up step nor the last timed one starts
    # anything ahead, so every copy of the timed steps is inside the region
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    # inputs prefetched and (MR_PIPELINE, default on) each next iteration's
    # map queued while this one is ordered, as bench.py's schedule
    eng.prefetch, eng.pipeline = True, TUNABLES.pipeline
    for w in range(args.warmup):
        res = eng.run_iteration(prefetch_next=w < args.warmup - 1, lookahead=args.warmup - 1 - w)
    D.barrier(device=device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = eng.run_iteration(prefetch_next=i < args.steps - 1, lookahead=args.steps - 1 - i)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    D.barrier(device=device)
    ms = 1000.0 * D.all_reduce_max(time.perf_counter() - t0, device) / max(1, args.steps)
    words = D.all_reduce_sum_int(res.distinct_keys, device)
    postings = D.all_reduce_sum_int(res.total_value, device)
    ok = full_ok = None
    if args.validate:
        full_ok = validate_full(eng, res, cdir, off, world, rank)
    if args.validate and world == 1:
        import importlib
        mod = importlib.import_module(M)
        with open(os.path.join(cdir, "blob.bin"), "rb") as f:
            blob = f.read(int(off[len(off) // 8]))
        sub = [blob[off[i]:off[i + 1]] for i in range(len(off) // 8)]
        e2 = spmd(dict(params, init_args={"nsplits": len(sub), "num_reducers": args.reducers}), device=device,
                  split_store=SplitStore(sub))
        e2.run()
        ok = mod.RESULT == mod.naive_index(sub)
    if rank == 0:
        print(f"# phases (last step, s): {res.timings}", file=sys.stderr)
        tokens = corpus.EUROPARL_WORDS
        print(json.dumps({
            "metric": "inverted-index build tokens/s (whole node), Europarl-v7-shaped 197 splits",
            "value": tokens / (ms / 1000.0), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
            "postings_per_s": postings / (ms / 1000.0), "distinct_words": words, "postings": postings,
            "validated_subset": ok, "validated_full": full_ok, "data": "synthetic Europarl-v7-shaped corpus, host-pinned, staged every step",
            "config": {"model": "examples/InvertedIndex (word -> sorted distinct line ids) on mr.spmd",
                       "parallelism": f"dp{world}", "num_reducers": args.reducers}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if (ok is not False and full_ok is not False) else 3


if __name__ == "__main__":
    sys.exit(main())
