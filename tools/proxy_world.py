#!/usr/bin/env python
"""Per-rank proxy of the W>1 SPMD iteration on ONE GPU: rank 0 of a simulated
world of N ranks maps its 1/N of the corpus and runs the whole multi-rank
path (compact -> FNV partition -> pack by destination -> count exchange ->
two all-to-alls -> reduce table -> fused tail -> host results) with the
collectives replaced by a loopback (every peer is assumed to send what this
rank sends: same volumes, no xGMI time).  Shows the device work and the host
overheads of the W>1 path that RCCL latency then adds to.

    python tools/proxy_world.py --world 8 [--steps 20]
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
from lua_mapreduce_1_amd.utils.config import TUNABLES  # noqa: E402
from lua_mapreduce_1_amd.parallel import spmd as S  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    _, _, device = D.init_from_env()
    splits = load_corpus(1234, 0, 0, 1, device)
    store = S.SplitStore(splits)
    W = a.world
    # loopback collectives: every peer sends this rank what this rank sends to
    # rank 0 (its own partitions) — the received volume and the distinct keys
    # after the reduce are those of a real rank of a W-rank job
    def exchange_counts(counts, group=None):
        c = counts.view(W, 3)
        return c[0:1].expand(W, 3).reshape(-1).clone()

    def all_to_all_v(payload, send, recv, group=None):
        return payload[:send[0]].repeat((W,) + (1,) * (payload.dim() - 1))
    D.exchange_counts = exchange_counts
    D.all_to_all_v = all_to_all_v
    S.D.world_info = lambda group=None: (0, W)
    params = dict(taskfn=MODEL, mapfn=MODEL, partitionfn=MODEL, reducefn=MODEL, finalfn=MODEL,
                  init_args={"nsplits": len(store), "num_reducers": 10})
    eng = S.SPMDEngine(params, device=device, split_store=store)
    assert eng.world == W and eng.rank == 0
    eng.prefetch = True
    eng.resident = os.environ.get("MR_RESIDENT") == "1"
    eng.pipeline = TUNABLES.pipeline  # MR_PIPELINE
    import gc
    gc_early = os.environ.get("MR_GC_EARLY", "1") == "1"  # as bench.py
    if gc_early:  # collect before the warm-up: the heap walk evicts the caches the timed steps run from
        gc.collect()
        gc.freeze()
    for w in range(a.warmup):
        eng.run_iteration(prefetch_next=w < a.warmup - 1, lookahead=a.warmup - 1 - w)
    if not gc_early:
        gc.collect()
    gc.freeze()
    torch.cuda.synchronize()
    if os.environ.get("MR_HOT_CPU"):  # diagnosis only: is the first timed step slow because the core idled?
        t_hot = time.perf_counter() + float(os.environ["MR_HOT_CPU"]) * 1e-3
        while time.perf_counter() < t_hot:
            pass
    copy_ev = []
    if os.environ.get("MR_COPY_TIMELINE"):
        # diagnosis: timing events around every iteration's input copies on
        # the copy stream -> copy durations and the copy engine's idle gaps
        orig = eng._issue_copies

        def issue(plan, wait_for=None):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(eng.copy_stream)
            orig(plan, wait_for)
            e1.record(eng.copy_stream)
            copy_ev.append((e0, e1, time.perf_counter()))
        eng._issue_copies = issue
    per = []
    prof = None
    if os.environ.get("MR_CPROFILE"):
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    from lua_mapreduce_1_amd.ops import _hip
    if _hip.WAIT_LOG is not None:
        _hip.WAIT_LOG.clear()
    t0 = time.perf_counter()
    prof_at = {int(x) for x in os.environ.get("MR_CPROFILE_ITERS", "").split(",") if x}
    for i in range(a.steps):
        t1 = time.perf_counter()
        if i in prof_at:  # cProfile of single iterations (first timed vs steady state)
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        res = eng.run_iteration(prefetch_next=i < a.steps - 1, lookahead=a.steps - 1 - i)
        per.append(1000 * (time.perf_counter() - t1))
        if i in prof_at:
            pr.disable()
            print(f"== cProfile of timed iteration {i}", file=sys.stderr)
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(18)
        if os.environ.get("MR_PHASES") and i < 3:
            print(i, {k: round(1000 * v, 3) for k, v in res.timings.items()}, file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / a.steps
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats(os.environ.get("MR_CPROFILE_SORT", "tottime")).print_stats(45)
    if _hip.WAIT_LOG is not None:
        for ta, tb, ok in _hip.WAIT_LOG[:12]:
            print(f"wait_stream at {1e6 * (ta - t0):9.1f} us: {1e6 * (tb - ta):7.1f} us (flag seen {ok})",
                  file=sys.stderr)
    from lua_mapreduce_1_amd.utils import trace
    if trace.LOG is not None:
        its = [e for e in trace.LOG if e[0] == "mr.iteration" and e[1] >= t0]
        for k in (0, 1, len(its) // 2):
            a, b = its[k][1], its[k][2]
            print(f"-- host timeline of timed iteration {k} ({1e6 * (b - a):.1f} us)", file=sys.stderr)
            for name, s0, s1 in sorted((e for e in trace.LOG if a <= e[1] <= b), key=lambda e: e[1]):
                print(f"   {1e6 * (s0 - a):8.1f} +{1e6 * (s1 - s0):7.1f}  {name}", file=sys.stderr)
    if copy_ev:
        c = copy_ev[-30:]
        dur = [round(a.elapsed_time(b), 3) for a, b, _ in c]
        gap = [round(c[i][1].elapsed_time(c[i + 1][0]), 3) for i in range(len(c) - 1)]
        per_it = [round(c[i][0].elapsed_time(c[i + 1][0]), 3) for i in range(len(c) - 1)]
        print(f"copies (last {len(c)}): duration ms {dur}", file=sys.stderr)
        print(f"copy engine idle gap ms {gap}", file=sys.stderr)
        print(f"copy start-to-start ms {per_it}", file=sys.stderr)
        print(f"host issue spacing ms {[round(1e3 * (c[i + 1][2] - c[i][2]), 3) for i in range(len(c) - 1)]}",
              file=sys.stderr)
    seq = [round(x, 2) for x in per]
    per.sort()
    print(json.dumps({"world": W, "ms_per_step": ms, "median": per[len(per) // 2], "min": per[0], "seq": seq,
                      "distinct_after_reduce": res.distinct_keys, "timings": res.timings}), flush=True)
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.exit(rc)
