"""Why is the first timed iteration slow?  Times the phases of consecutive
iterations of the 1/N per-rank proxy with host timestamps and CUDA events."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import MODEL, load_corpus  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel import spmd as S  # noqa: E402

_, _, device = D.init_from_env()
splits = load_corpus(1234, 0, 0, 1, device)
k = (len(splits) + 7) // 8
store = S.SplitStore(splits[:k])
eng = S.SPMDEngine(dict(taskfn=MODEL, mapfn=MODEL, partitionfn=MODEL, reducefn=MODEL, finalfn=MODEL,
                        init_args={"nsplits": k, "num_reducers": 10}), device=device, split_store=store)
orig_run_map = eng._run_map
orig_stats = eng.tables[0].stats.__func__


def timed_run_map(*a, **kw):
    t = time.perf_counter()
    orig_run_map(*a, **kw)
    print(f"    run_map issue {1000 * (time.perf_counter() - t):.3f} ms", flush=True)


eng._run_map = timed_run_map


def slow_wrap(obj, name):
    f = getattr(obj, name)

    def w(*a, **kw):
        t = time.perf_counter()
        r = f(*a, **kw)
        dt = 1000 * (time.perf_counter() - t)
        if dt > 1.0:
            print(f"      SLOW {name}: {dt:.3f} ms", flush=True)
        return r
    setattr(obj, name, w)


from lua_mapreduce_1_amd.ops import _hip as H  # noqa: E402
from lua_mapreduce_1_amd import ops as O  # noqa: E402
slow_wrap(eng, "_issue_copies")
slow_wrap(H, "call")
slow_wrap(O.HashTable, "_overflow")
slow_wrap(O.HashTable, "reset")
slow_wrap(O.HashTable, "stats")
slow_wrap(torch.cuda.Stream, "wait_event")
slow_wrap(torch.cuda.Event, "query")
import gc
_gc_t = [0.0]


def _gc_cb(phase, info):
    if phase == "start":
        _gc_t[0] = time.perf_counter()
    elif info["generation"] == 2:
        print(f"    gen2 GC {1000 * (time.perf_counter() - _gc_t[0]):.3f} ms, collected {info['collected']}", flush=True)


gc.callbacks.append(_gc_cb)
if os.environ.get("MR_FREEZE"):
    gc.collect()
    gc.freeze()
if os.environ.get("MR_PRIME"):
    # prime the copy path: a few rounds of the real chunk copies behind a
    # cross-stream wait, before any iteration
    ids = list(range(k))
    for r in range(int(os.environ["MR_PRIME"])):
        t = time.perf_counter()
        plan = eng._get_plan(ids, r % 2)
        eng._issue_copies(plan, wait_for=torch.cuda.current_stream())
        eng.copy_stream.synchronize()
        print(f"  prime {r}: {1000 * (time.perf_counter() - t):.3f} ms", flush=True)
for i in range(int(os.environ.get('MR_ITERS', 8))):
    if i == 4:
        time.sleep(0.5)
        print("  (slept 0.5 s)")
    torch.cuda.synchronize()
    t = time.perf_counter()
    if i == 2 and os.environ.get("MR_CPROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        r = eng.run_iteration(prefetch_next=False)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(12)
    else:
        r = eng.run_iteration(prefetch_next=False)
    print(f"iter {i}: {1000 * (time.perf_counter() - t):.3f} ms {({k: round(1000 * v, 3) for k, v in r.timings.items()})}",
          flush=True)
