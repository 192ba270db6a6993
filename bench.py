#!/usr/bin/env python
"""Headline benchmark: Europarl-v7-shaped word-count, words/s for the whole node.

Workload (BASELINE.json / BASELINE.md; reference README.md:43-75): 197 input
splits of <=10,000 lines, 1,965,734 lines and 49,158,635 whitespace tokens
(synthetic, Zipf-Mandelbrot vocabulary, ~291 MB — no network for the real
corpus), one map job per split, sum reducer used as combiner, 10 reduce
partitions (README.md:59).

One timed step = one full MapReduce iteration through the SPMD engine
(parallel/spmd.py): taskfn -> host(pinned) -> HBM staging of every split ->
fused tokenize/key/combine kernels -> partition -> RCCL all-to-all shuffle
(N>1) -> per-partition reduce -> (partition, key) radix sort -> key bytes +
counts of every ``result.P<NN>`` copied back to host memory.  As in the
reference's "Server time" (server.lua:464-536), the user finalfn that prints
results is not part of the step; it runs once after timing to validate.

Before the steady-state steps, ONE cold iteration is timed from the split
files on disk (page cache dropped with posix_fadvise, best effort) to the
results in host memory — the shape of the reference's single 49 s run, whose
mapfns read their split files (examples/WordCount/mapfn.lua:4).  It is
reported as ``cold_first_iteration_ms`` next to the steady-state headline.
Every rank reads and pins only its own splits (native loader, ops/io.py).

The corpus is fixed, so adding GPUs divides it (strong scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--from-files DIR]

With N > 1 and no torchrun environment, the script starts the N ranks itself
(``python -m torch.distributed.run --nproc-per-node N ...`` as a child process;
rank 0's JSON line is relayed on stdout, the exit code is the launcher's).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
BASELINE_WORDS_PER_S = 49_158_635 / 49.229152  # README.md:73 (4 workers, 1 machine)
METRIC = "words/sec (whole node), Europarl-v7 word-count 197 splits, 1/2/4/8 MI355X"
MODEL = "lua_mapreduce_1_amd.models.wordcount"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--reducers", type=int, default=10)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--resident", action="store_true",
                    help="keep the corpus in HBM across steps (default: stage it from host memory every step)")
    ap.add_argument("--from-files", default=None, metavar="DIR",
                    help="corpus = the files in DIR (sorted; one split per file) instead of the synthetic one")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold file-to-result first iteration")
    ap.add_argument("--force-shuffle", action="store_true",
                    help="also time the W>1 data path (pack, count exchange, RCCL all_to_all_single, receive-side "
                         "reduce) at one GPU: a one-rank nccl group, reported as force_shuffle_ms_per_step")
    # smaller corpora only for smoke tests of the harness (the headline number
    # is the full Europarl shape; a reduced one is flagged in "data"/"config")
    ap.add_argument("--lines", type=int, default=None)
    ap.add_argument("--words", type=int, default=None)
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """Start n ranks of this script under torchrun (a child process: nothing
    here has touched the GPU) and return the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    try:
        r = subprocess.run(cmd, env=env, cwd=ROOT)
    except OSError as e:
        print(f"# could not start {n} ranks: {e}", file=sys.stderr)
        return 2
    if r.returncode != 0:
        print(f"# rank launcher exited with {r.returncode}", file=sys.stderr)
    return r.returncode


# ---------------------------------------------------------------------------
def corpus_dir(seed: int, lines: int, words: int) -> str:
    from lua_mapreduce_1_amd.utils import corpus
    shape = "" if (lines, words) == (corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS) else f"_{lines}_{words}"
    return f"/tmp/lmr_europarl_like_{seed}{shape}"


def ensure_corpus(d: str, seed: int, lines: int, words: int) -> None:
    """Generate once per box: blob.bin + off.npy (splits back to back), the
    split files files/split%05d.txt, and the per-word ground truth."""
    import numpy as np
    from lua_mapreduce_1_amd.utils import corpus
    if os.path.exists(os.path.join(d, "done")):
        return
    t0 = time.time()
    splits, vocab, counts = corpus.europarl_like(seed=seed, lines=lines, words=words, return_counts=True)
    tmp = d + f".tmp{os.getpid()}"
    os.makedirs(tmp, exist_ok=True)
    off = np.zeros(len(splits) + 1, np.int64)
    np.cumsum([len(s) for s in splits], out=off[1:])
    with open(os.path.join(tmp, "blob.bin"), "wb") as f:
        for s in splits:
            f.write(s)
    np.save(os.path.join(tmp, "off.npy"), off)
    corpus.write_splits(splits, os.path.join(tmp, "files"))
    keep = counts > 0
    vb = [w for w, k in zip(vocab, keep) if k]
    voff = np.zeros(len(vb) + 1, np.int64)
    np.cumsum([len(w) for w in vb], out=voff[1:])
    np.save(os.path.join(tmp, "vocab_off.npy"), voff)
    np.save(os.path.join(tmp, "vocab_counts.npy"), counts[keep])
    with open(os.path.join(tmp, "vocab.bin"), "wb") as f:
        f.write(b"".join(vb))
    open(os.path.join(tmp, "done"), "w").close()
    if os.path.exists(d):
        import shutil
        shutil.rmtree(d, ignore_errors=True)
    os.replace(tmp, d)
    print(f"# corpus generated in {time.time() - t0:.1f}s -> {d}", file=sys.stderr, flush=True)


def load_corpus(seed: int = 1234, lines: int = 0, words: int = 0, *_unused) -> list:
    """The synthetic corpus's splits as a list of bytes (generated and cached
    as the benchmark does; 0 = the Europarl shape).  For tools/."""
    import numpy as np
    from lua_mapreduce_1_amd.utils import corpus
    lines = lines or corpus.EUROPARL_LINES
    words = words or corpus.EUROPARL_WORDS
    d = corpus_dir(seed, lines, words)
    ensure_corpus(d, seed, lines, words)
    off = np.load(os.path.join(d, "off.npy"))
    with open(os.path.join(d, "blob.bin"), "rb") as f:
        blob = f.read()
    return [blob[off[i]:off[i + 1]] for i in range(off.size - 1)]


def truth_counts(d: str) -> dict:
    import numpy as np
    voff = np.load(os.path.join(d, "vocab_off.npy"))
    cnt = np.load(os.path.join(d, "vocab_counts.npy"))
    with open(os.path.join(d, "vocab.bin"), "rb") as f:
        vb = f.read()
    return {vb[voff[i]:voff[i + 1]]: int(cnt[i]) for i in range(cnt.size)}


def result_counts(eng, res) -> dict:
    """word -> count from every rank's result partitions (on rank 0)."""
    import numpy as np
    out = {}
    for _name, cols in eng.gather_results(res):
        off, blob, val = cols["key_off"], cols["key_blob"], cols["val"]
        b = blob.tobytes() if isinstance(blob, np.ndarray) else bytes(blob)
        for i in range(val.size):
            out[b[int(off[i]):int(off[i + 1])]] = int(val[i])
    return out


def main() -> int:
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)

    import gc

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from lua_mapreduce_1_amd.parallel import dist as D
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils import corpus
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    from lua_mapreduce_1_amd.ops import io as mio

    lines = args.lines or corpus.EUROPARL_LINES
    words = args.words or corpus.EUROPARL_WORDS
    rank, world, device = D.init_from_env()
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if device.type == "cuda":
        # host buffers (pinned splits, downloads) on the GPU's own socket
        from lua_mapreduce_1_amd.utils import numa
        nb = numa.bind_to_gpu(device.index or 0)
        if args.verbose or rank == 0:
            print(f"# rank {rank}: GPU {nb['pci']} on NUMA node {nb['node']}, {nb['cpus']} CPUs bound",
                  file=sys.stderr, flush=True)
    import torch.distributed as dist
    backend = dist.get_backend() if dist.is_initialized() else ("single-process-" + device.type)
    if args.force_shuffle and world == 1 and not dist.is_initialized():
        # a one-rank group, created before any other GPU work: the shuffle's
        # collectives then run on RCCL (nccl backend) as at W > 1
        import datetime
        kw = {"device_id": device} if device.type == "cuda" else {}
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo", rank=0, world_size=1,
                                init_method=f"tcp://127.0.0.1:{_free_port()}",
                                timeout=datetime.timedelta(seconds=300), **kw)
    if world != args.gpus and rank == 0:
        print(f"# warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if device.type == "cuda":
        torch.zeros(1, device=device)  # context creation is process start-up, not part of any iteration
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)

    if args.from_files:
        import glob
        paths = sorted(p for p in glob.glob(os.path.join(args.from_files, "*")) if os.path.isfile(p))
        cdir = None
        full = False
    else:
        cdir = corpus_dir(args.seed, lines, words)
        if local_rank == 0:
            ensure_corpus(cdir, args.seed, lines, words)
        D.barrier(device=device)
        paths = sorted(os.path.join(cdir, "files", f) for f in os.listdir(os.path.join(cdir, "files")))
        full = (lines, words) == (corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
    params = dict(taskfn=MODEL, mapfn=MODEL, partitionfn=MODEL, reducefn=MODEL, finalfn=MODEL,
                  init_args={"nsplits": len(paths), "num_reducers": args.reducers})

    # -- one cold iteration: split files on disk -> results in host memory ----
    cold_ms = None
    cold_tokens = None
    table_cap = 1 << 20
    store = None
    if not args.no_cold:
        dropped = all(mio.drop_page_cache(p) for p in paths)
        D.barrier(device=device)
        sync()
        t0 = time.perf_counter()
        store = SplitStore.from_files(paths, rank, world, pin=device.type == "cuda")
        eng = SPMDEngine(params, device=device, split_store=store, verbose=args.verbose)
        eng.prime_plans = False
        res = eng.run_iteration(prefetch_next=False)
        sync()
        cold = time.perf_counter() - t0
        D.barrier(device=device)
        cold_ms = 1000.0 * D.all_reduce_max(cold, device)
        cold_tokens = D.all_reduce_sum_int(res.total_value, device)
        table_cap = eng._table_capacity  # sized from the cold map's distinct keys (MR_MAP_SPARSITY)
        del eng, res
        store.finish_loading()
    if store is None:
        if cdir is not None:
            store = SplitStore.from_blob(os.path.join(cdir, "blob.bin"), np.load(os.path.join(cdir, "off.npy")),
                                         rank, world, pin=device.type == "cuda")
        else:
            store = SplitStore.from_files(paths, rank, world, pin=device.type == "cuda")
        store.finish_loading()
    total_bytes = int(store.offsets[-1])

    eng = SPMDEngine(params, device=device, split_store=store, verbose=args.verbose, table_capacity=table_cap)
    # consecutive iterations are pipelined: the next iteration's input copies
    # start as soon as the HBM arena they fill is free (double-buffered), and
    # its map as soon as this map is done; neither the last warm-up step nor
    # the last timed step starts anything for the next one, so the timed
    # region holds exactly `steps` iterations of work (and one pipeline fill)
    eng.prefetch = True
    # --resident: the corpus stays in HBM across steps —
    # a different measurement from the default, which re-reads the input from
    # host memory every step as the reference re-reads its split files
    eng.resident = args.resident
    # ... and pipelined: iteration i+1's map runs on a second stream while
    # iteration i shuffles, reduces and downloads its results
    eng.pipeline = TUNABLES.pipeline  # MR_PIPELINE
    # long-lived objects (modules, corpus, engine) move to the permanent GC
    # generation: a full collection over them stalled an iteration by ~5 ms
    # every few dozen iterations.  Collected BEFORE the warm-up: the heap walk
    # evicts the CPU caches, and right before the timed region it made the
    # first step's host work 2-4x slower
    gc.collect()
    gc.freeze()
    for w in range(args.warmup):
        eng.run_iteration(prefetch_next=w < args.warmup - 1, lookahead=args.warmup - 1 - w)
    gc.freeze()  # the warm-up's survivors too (no heap walk)
    D.barrier(device=device)
    sync()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = eng.run_iteration(prefetch_next=i < args.steps - 1, lookahead=args.steps - 1 - i)
    if hasattr(last, "wait"):
        last.wait()  # the last step's result columns are in host memory (a lazy download landed)
    sync()
    D.barrier(device=device)
    elapsed = time.perf_counter() - t0
    elapsed = D.all_reduce_max(elapsed, device)
    ms = 1000.0 * elapsed / max(1, args.steps)

    # validation outside the timed region: every token counted exactly once,
    # and (synthetic corpus) every word's count equal to the generator's (read
    # before any other engine runs: result columns live in the pinned
    # download buffers until the next tail)
    counted = D.all_reduce_sum_int(last.total_value, device) if last is not None else 0
    distinct = D.all_reduce_sum_int(last.distinct_keys, device) if last is not None else 0
    got = result_counts(eng, last) if last is not None else {}

    fs_ms = fs_valid = None
    if args.force_shuffle:
        # the same steps with the W > 1 path forced at this world size
        e2 = SPMDEngine(dict(params, force_shuffle=True), device=device, split_store=store, verbose=args.verbose,
                        table_capacity=table_cap)
        e2.prefetch, e2.resident, e2.pipeline = True, args.resident, TUNABLES.pipeline
        for w in range(args.warmup):
            e2.run_iteration(prefetch_next=w < args.warmup - 1, lookahead=args.warmup - 1 - w)
        D.barrier(device=device)
        sync()
        t0 = time.perf_counter()
        r2 = None
        for i in range(args.steps):
            r2 = e2.run_iteration(prefetch_next=i < args.steps - 1, lookahead=args.steps - 1 - i)
        if hasattr(r2, "wait"):
            r2.wait()
        sync()
        D.barrier(device=device)
        fs_ms = 1000.0 * D.all_reduce_max(time.perf_counter() - t0, device) / max(1, args.steps)
        fs_valid = r2 is not None and D.all_reduce_sum_int(r2.total_value, device) == words
        del e2, r2

    per_key = None
    if rank == 0 and cdir is not None:
        per_key = got == truth_counts(cdir)
    if cdir is None:
        words = counted  # external files: the engine's own token count
    block = eng.stats_block(last) if last is not None else ""  # a collective at W > 1: every rank
    valid = True
    if rank == 0:
        print(block, file=sys.stderr, end="")
        print(f"# tokens counted {counted} (expected {words}), distinct words {distinct}, per-key match {per_key}, "
              f"bytes {total_bytes}, per-phase s: {last.timings}, cold first iteration ms {cold_ms} "
              f"(tokens {cold_tokens}, page cache dropped {not args.no_cold and dropped})",
              file=sys.stderr, flush=True)
        valid = counted == words and per_key is not False and (cold_tokens is None or cold_tokens == words) and \
            fs_valid is not False
        if not valid:
            print("# ERROR: result validation failed", file=sys.stderr, flush=True)
        value = words / (ms / 1000.0)
        out = {
            "metric": METRIC, "value": value, "unit": "words/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": value / BASELINE_WORDS_PER_S, "dtype": "int64",
            "data": (("synthetic Europarl-v7-shaped corpus" if cdir else f"files in {args.from_files}")
                     + f" ({len(store)} splits, {lines:,} lines, {words:,} words, {total_bytes} bytes)"
                     + ("" if full or not cdir else " REDUCED (smoke test only)")
                     + (", HBM-resident splits (copied to HBM once, before timing; --resident)" if args.resident
                        else ", host-resident pinned splits staged to HBM every step (later steps' copies overlap "
                        "this step's map/reduce)")),
            "backend": backend, "world": world,
            "cold_first_iteration_ms": cold_ms,
            **({"force_shuffle_ms_per_step": fs_ms, "force_shuffle_valid": fs_valid,
                "force_shuffle_backend": dist.get_backend() if dist.is_initialized() else None}
               if args.force_shuffle else {}),
            "config": {"model": "wordcount (MapReduce: taskfn/mapfn/partitionfn/reducefn)", "global_batch": len(store),
                       "seq_len": 10000, "parallelism": f"dp{world}", "num_reducers": args.reducers,
                       "words": words, "bytes": total_bytes, "valid": valid, "per_key_valid": per_key,
                       "input": "hbm-resident" if args.resident else "host-staged-every-step"},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    # a wrong answer is a failed run: the driver's exit code sees it
    return 0 if valid else 3


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    if os.environ.get("MR_FAST_EXIT"):
        os._exit(rc)  # skip library finalizers (seen to segfault under rocprofv3 --memory-copy-trace)
    sys.exit(rc)
