#!/usr/bin/env python
"""Throughput of user device maps that pick their own keys (byte spans,
``ops/text.py``) through the MapReduce API on mr.spmd — the general plane
(parallel/generic.py: typed folds, value lists) and, for an int64 ``sum``,
the fold plane:

* bigram: examples/Bigram (byte-span keys = two consecutive tokens of a
  line, int64 sum) over bench.py's Europarl-shaped corpus (197 splits,
  291 MB, ~47 M bigrams);
* scores: examples/ScoreStats (CSV ``word,score``: field split + decimal
  parse in one fused kernel, typed f64 mean / f64 max / count folds) over a generated
  CSV (``--score-lines`` lines).

* wc_general: word count with the reference's GENERAL reducer contract
  (examples/WordCount/reducefn2: sum, combinerfn = reducefn, no ACI flags,
  no device_reduce) over the Europarl-shaped corpus — the host combiner and
  reducer (``reducefn2``) and their batched device form (``reducefn3``:
  device_reducefn) — reporting the values left after the map-side combine
  (what a rank would ship) next to the 49 M emitted.

Input is staged from pinned host memory every step, like the headline.  The
first warm-up iteration of each job is checked against the module's naive
oracle on a subset of splits (exact equality; float means within 1e-9);
``--validate`` also checks the LAST timed step's full result, every key,
against the generator's ground truth (``validated_full``).  Prints one JSON
line per job.

    python tools/bench_generic.py [--steps K] [--warmup W] [--jobs bigram,scores,wc_general] [--validate]
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
    if hasattr(res, "wait"):
        res.wait()  # inside the clock: the last step's results landed in host memory
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


def result_pairs(eng, res) -> dict:
    """key bytes -> values (a list) of every partition of a result."""
    from lua_mapreduce_1_amd.runtime import codec
    out = {}
    for _name, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            out[k] = v
    return out


def run_job(name: str, mod_name: str, store, nbytes: int, check_splits: list[bytes] | None, units: int, unit: str,
            args, device, params: dict | None = None, truth=None) -> dict:
    """``params``: module names (default: every function from ``mod_name``);
    ``truth``: callable(result dict) -> bool, the full per-key check run on
    the last timed step's result with ``--validate``."""
    M = mod_name
    p = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M)
    p.update(params or {})
    p["init_args"] = {"nsplits": len(store), "num_reducers": 10, "quiet": True}
    eng = spmd(p, device=device, split_store=store)
    ms, res = _time(eng, args.steps, args.warmup, device)
    # read the result before the check runs another engine (result columns
    # alias the process's pinned download buffers until the next tail)
    out = {"metric": f"{name} {unit}/s (device_mapfn with span emits, mr.spmd)", "value": units / (ms / 1000.0),
           "unit": f"{unit}/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
           "bytes": int(nbytes), "GB_per_s": nbytes / (ms / 1000.0) / 1e9, "distinct_keys": res.distinct_keys,
           "total_value": res.total_value, "timings_last_step": res.timings}
    mp = getattr(eng.plane, "map", None)
    # the map tables' capacities (slots): the reset and the compaction stream every slot
    caps = [int(t.cap) for t in getattr(eng, "tables", []) if t is not None]
    for m in getattr(eng.plane, "_maps", None) or []:
        if getattr(m, "table", None) is not None:
            caps.append(int(m.table.cap))
    if getattr(mp, "table", None) is not None:
        caps.append(int(mp.table.cap))
    out["table_caps"] = sorted(set(caps))
    if getattr(mp, "reducers", None) is not None:
        out["combines_last_step"] = mp.combines
        out["values_after_combine"] = int(mp.table.npost)
        out["values_emitted"] = int(mp.rows)
        out["recognized_folds"] = dict(mp.reducers.recognized)
    if args.validate and truth is not None:
        t0 = time.time()
        out["validated_full"] = bool(truth(result_pairs(eng, res)))
        out["validate_s"] = time.time() - t0
    del res
    if check_splits is not None:
        out["oracle_subset_ok"] = _check(mod_name, check_splits, device)
    return out


def _bigram_truth(cdir: str):
    """(vocab, codes, counts) of the corpus's bigrams, cached next to it."""
    f = os.path.join(cdir, "bigram_truth.npz")
    if not os.path.exists(f):
        t0 = time.time()
        _s, vocab, _c, (codes, cnt) = corpus.europarl_like(seed=1234, return_bigrams=True)
        voff = np.zeros(len(vocab) + 1, np.int64)
        np.cumsum([len(w) for w in vocab], out=voff[1:])
        np.savez(f + ".tmp.npz", codes=codes, counts=cnt, voff=voff,
                 vocab=np.frombuffer(b"".join(vocab), np.uint8))
        os.replace(f + ".tmp.npz", f)
        print(f"# bigram truth computed in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    z = np.load(f)
    vb = z["vocab"].tobytes()
    voff = z["voff"]
    vocab = [vb[voff[i]:voff[i + 1]] for i in range(voff.size - 1)]
    return vocab, z["codes"], z["counts"]


def _check_bigrams(cdir: str, got: dict) -> bool:
    vocab, codes, cnt = _bigram_truth(cdir)
    V = len(vocab)
    if len(got) != codes.size:
        print(f"# bigram validation: {len(got)} keys, truth {codes.size}", file=sys.stderr)
        return False
    vid = {w: i for i, w in enumerate(vocab)}
    gc = np.empty(len(got), np.int64)
    gv = np.empty(len(got), np.int64)
    for j, (k, v) in enumerate(got.items()):
        b = k.encode("utf-8", "surrogateescape")
        i = b.index(b" ")
        gc[j] = vid[b[:i]] * V + vid[b[i + 1:]]
        gv[j] = v[0]
    o = np.argsort(gc)
    return bool(np.array_equal(gc[o], codes) and np.array_equal(gv[o], cnt))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--jobs", default="bigram,scores")
    ap.add_argument("--score-lines", type=int, default=8_000_000)
    ap.add_argument("--wc-reducers", default="reducefn3,reducefn2",
                    help="wc_general: the WordCount reduce modules to run")
    ap.add_argument("--validate", action="store_true",
                    help="check every key of the last timed step against the generator's ground truth")
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
                      "bigrams", args, device, truth=lambda got: _check_bigrams(cdir, got))
        out["bigrams_expected"] = bigrams
        out["bigrams_counted"] = out["total_value"]
        rc |= 0 if (out["oracle_subset_ok"] and out["total_value"] == bigrams and
                    out.get("validated_full", True)) else 3
        print(json.dumps(out), flush=True)
    if "scores" in jobs:
        t0 = time.time()
        splits, stru = corpus.score_csv(seed=11, lines=args.score_lines, vocab_size=300_000,
                                        split_lines=max(1, args.score_lines // 197), return_truth=True)
        print(f"# generated {args.score_lines} CSV lines in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        out = run_job("CSV group-by mean/max/count", "lua_mapreduce_1_amd.examples.ScoreStats", SplitStore(splits),
                      sum(len(x) for x in splits), splits[:4], args.score_lines, "rows", args, device,
                      truth=lambda got: got.keys() == stru.keys() and all(_close(got[k], stru[k]) for k in stru))
        rc |= 0 if (out["oracle_subset_ok"] and out.get("validated_full", True)) else 3
        print(json.dumps(out), flush=True)
    if "wc_general" in jobs:
        cdir = corpus_dir(1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
        ensure_corpus(cdir, 1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
        from bench import truth_counts
        off = np.load(os.path.join(cdir, "off.npy"))
        store = SplitStore.from_blob(os.path.join(cdir, "blob.bin"), off)
        store.finish_loading()
        tc = {k.decode("utf-8", "surrogateescape"): v for k, v in truth_counts(cdir).items()}
        W = "lua_mapreduce_1_amd.models.wordcount"
        for red in args.wc_reducers.split(","):
            a = argparse.Namespace(**vars(args))
            from lua_mapreduce_1_amd.utils.config import TUNABLES
            if red == "reducefn2" and not TUNABLES.recognize_reducers:
                a.steps, a.warmup = min(args.steps, 2), 1  # per-key Python combiner + reducer: seconds per step
            out = run_job(f"word count, general reducer {red}", W, store, int(off[-1]), None,
                          corpus.EUROPARL_WORDS, "words", a, device,
                          params={"reducefn": "lua_mapreduce_1_amd.examples.WordCount." + red},
                          truth=lambda got: got.keys() == tc.keys() and all(got[k] == [tc[k]] for k in tc))
            out["values_emitted_expected"] = corpus.EUROPARL_WORDS
            ok = out["total_value"] == corpus.EUROPARL_WORDS and out.get("validated_full", True) and \
                out.get("values_after_combine", 0) <= out["distinct_keys"]
            rc |= 0 if ok else 3
            print(json.dumps(out), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
