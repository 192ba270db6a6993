"""CPU simulation of the map kernel's HBM flush count on the synthetic Europarl token stream: per-chunk
combine at several chunk sizes, and persistent workgroup spans with a capped, evicting LDS table
(profiles/r2/map_kernel/flush_simulation.txt)."""
import numpy as np, sys
sys.path.insert(0, '.')
from lua_mapreduce_1_amd.utils import corpus as C
# regenerate token ids stream quickly (same distribution as europarl_like)
rng = np.random.default_rng(1234)
V=300_000
cdf = np.cumsum(C.zipf_probs(V)); cdf[-1]=1
N = 6_000_000   # 1/8 of corpus worth of tokens
tok = np.minimum(np.searchsorted(cdf, rng.random(N), side="right"), V-1)
# ~5.93 bytes per token -> 8KB chunk ~ 1380 tokens
def per_chunk(ct):
    n=0
    for a in range(0, N, ct):
        n += np.unique(tok[a:a+ct]).size
    return n
for ct in (1380, 2760, 11000, 44000):
    print("chunk tokens", ct, "flushes/token %.3f" % (per_chunk(ct)/N))
# persistent WG with LDS capacity C, span S tokens, policy: when full (C distinct), flush entries with count<=k and keep the rest
def persistent(span, Cap, keep_thr):
    flushes=0
    for a in range(0, N, span):
        seg = tok[a:a+span]
        table = {}
        for t in seg:
            table[t] = table.get(t,0)+1
            if len(table) >= Cap:
                drop = [k for k,v in table.items() if v <= keep_thr]
                if len(drop) < Cap//4:
                    drop = list(table.keys())
                flushes += len(drop)
                for k in drop: del table[k]
        flushes += len(table)
    return flushes
for span, cap, thr in ((96000, 3072, 1), (96000, 3072, 2), (96000,1536,1), (24000, 3072, 1)):
    f = persistent(span, cap, thr)
    print("persistent span", span, "cap", cap, "thr", thr, "flushes/token %.3f" % (f/N)) 
