"""Debug: forced sort give-up in the fused tail after the sort-only give-up test."""
import sys
from collections import Counter
import numpy as np
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.parallel import spmd as S
from lua_mapreduce_1_amd.runtime import device as devmod, codec
from lua_mapreduce_1_amd.utils.corpus import europarl_like

gpu = torch.device("cuda", 0)
mode = sys.argv[1]
if "pre" in mode:
    rng = np.random.default_rng(5)
    w = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, 300_000, dtype=np.int64))
    ops.debug_sort_fail(1); ops.sort_keys([w.to(gpu)]); print("err", ops.sort_error(gpu))
    ops.debug_sort_fail(1); ops.sort_keys_checked([w.to(gpu)])
    ops.debug_sort_fail(100)
    try:
        ops.sort_keys_checked([w.to(gpu)], retries=2)
    except RuntimeError as e:
        print("raised", e)
    ops.debug_sort_fail(0)
splits = europarl_like(seed=4, lines=20_000, words=300_000, vocab_size=30_000, split_lines=2000)
want = Counter(w.decode() for s in splits for w in s.split())
M = "lua_mapreduce_1_amd.models.wordcount"
orig = devmod.finalize
def spy(hi, lo, val, rep, src, nparts, pm=None, part=None, _presorted=False, need_keys=False):
    torch.cuda.synchronize()
    print("fallback finalize: n", hi.numel(), "val sum", int(val.sum()), "part sorted",
          bool((part[1:] >= part[:-1]).all()), "keys sorted?", flush=True)
    return orig(hi, lo, val, rep, src, nparts, pm, part, _presorted, need_keys)
devmod.finalize = spy
eng = S.SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                        init_args={"nsplits": len(splits), "num_reducers": 7}),
                   split_store=S.SplitStore(splits), device=gpu)
if "fail" in mode:
    ops.debug_sort_fail(1)
res = eng.run_iteration()
got = {k: v[0] for _n, c in eng.gather_results(res) for k, v in codec.iter_columnar(c)}
bad = [(k, got.get(k), want[k]) for k in want if got.get(k) != want[k]]
print(mode, "n", len(got), "mismatch", len(bad), bad[:4], flush=True)
