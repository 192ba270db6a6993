"""cProfile of SPMD word-count iterations (host-side overheads)."""
import cProfile, pstats, sys, os, time
sys.path.insert(0, ".")
import numpy as np, torch
from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
from lua_mapreduce_1_amd.utils import corpus
cache = "/tmp/lmr_europarl_like_1234.npz"
if not os.path.exists(cache):
    splits = corpus.europarl_like(seed=1234)
    off = np.zeros(len(splits) + 1, np.int64); np.cumsum([len(s) for s in splits], out=off[1:])
    np.savez(cache, data=np.frombuffer(b"".join(splits), np.uint8), off=off)
z = np.load(cache); data, off = z["data"], z["off"]
splits = [data[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
OF = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # 1/OF of the splits (per-rank proxy)
splits = splits[:(len(splits) + OF - 1) // OF]
M = "lua_mapreduce_1_amd.models.wordcount"
eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, init_args={"nsplits": len(splits)}),
                 split_store=SplitStore(splits), device=torch.device("cuda", 0))
for _ in range(3): eng.run_iteration()
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(20): eng.run_iteration()
pr.disable()
print("ms/iter", (time.perf_counter() - t0) * 50)
st = pstats.Stats(pr); st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(30)
