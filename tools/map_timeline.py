#!/usr/bin/env python
"""Event timeline of the SPMD map phase on ONE GPU for 1/N of the corpus:
per chunk, H2D start/end (copy stream) and map kernel start/end (compute
stream), relative to the first copy.  Shows how well staging overlaps."""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import MODEL, load_corpus  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore  # noqa: E402

of = int(sys.argv[1]) if len(sys.argv) > 1 else 8
_, _, device = D.init_from_env()
splits = load_corpus(1234, 0, 0, 1, device)
k = (len(splits) + of - 1) // of
store = SplitStore(splits[:k])
eng = SPMDEngine(dict(taskfn=MODEL, mapfn=MODEL, partitionfn=MODEL, reducefn=MODEL, finalfn=MODEL,
                      init_args={"nsplits": k, "num_reducers": 10}), device=device, split_store=store)
for _ in range(3):
    eng.run_iteration()
torch.cuda.synchronize()
key = next(iter(eng._plans))
b_, v_, h_, e_ = eng._plans[key]
eng._plans[key] = (b_, v_, h_, [torch.cuda.Event(enable_timing=True) for _ in e_])
# instrument: wrap copy + map with events
jobs = eng._jobs()
evs = []
orig_copy = torch.Tensor.copy_
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
t0 = E()
t0.record(eng.copy_stream)
chunks = []
gen = eng._stage_chunks(jobs, 0, len(jobs))
for (a, b), data in gen:
    e1, e2 = E(), E()
    e1.record()
    eng.table.wordcount_map(data, rep_base=int(data.data_ptr() - eng.arena.data_ptr()))
    e2.record()
    chunks.append((data.numel(), e1, e2))
torch.cuda.synchronize()
plan = next(iter(eng._plans.values()))
for i, ev in enumerate(plan[3]):
    print(f"copy {i} done at {t0.elapsed_time(ev)*1000:8.1f} us")
for n, e1, e2 in chunks:
    print(f"chunk {n/1e6:7.2f} MB  kernel {t0.elapsed_time(e1)*1000:8.1f} -> {t0.elapsed_time(e2)*1000:8.1f} us"
          f"  ({(t0.elapsed_time(e2)-t0.elapsed_time(e1))*1000:7.1f} us, "
          f"{n/((t0.elapsed_time(e2)-t0.elapsed_time(e1))/1000)/1e9:6.1f} GB/s)")
