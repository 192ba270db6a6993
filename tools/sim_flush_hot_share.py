"""CPU simulation on the synthetic Europarl token stream (6 M tokens): flush entries per token of the
map kernel's per-chunk combine, and the share of them that belongs to the top-K words (the case for a
static hot dictionary; profiles/r2/map_kernel/flush_simulation.txt)."""
import numpy as np, sys
sys.path.insert(0, '.')
from lua_mapreduce_1_amd.utils import corpus as C
rng = np.random.default_rng(1234)
V=300_000
cdf = np.cumsum(C.zipf_probs(V)); cdf[-1]=1
N = 6_000_000
tok = np.minimum(np.searchsorted(cdf, rng.random(N), side="right"), V-1)
ct=1380
tot=0; hot={k:0 for k in (256,1024,2048,4096,8192)}
for a in range(0, N, ct):
    u = np.unique(tok[a:a+ct]); tot += u.size
    for k in hot: hot[k] += int((u < k).sum())
print("flush entries per token %.3f" % (tot/N))
for k,v in hot.items(): print("top", k, "share of flush entries %.3f" % (v/tot))
