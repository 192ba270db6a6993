import sys; sys.path.insert(0, ".")
import numpy as np, torch
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.runtime import device as dv
from lua_mapreduce_1_amd.utils.corpus import tricky_text
gpu = torch.device("cuda:0")
nparts = 1
rng = np.random.default_rng(nparts)
text = tricky_text(rng, 400_000) + b" " + b" ".join(
    bytes(rng.integers(97, 123, int(rng.integers(1, 24))).astype(np.uint8)) for _ in range(20000)) + b"\n"
t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
tab = ops.HashTable(1 << 16, device=gpu)
tab.wordcount_map(t)
n, _ = tab.stats()
pend = dv.finalize_table_device(tab, n, t, nparts)
raw = dv._unpack_fused(pend) if False else None
a = dv.finalize_host(pend)
a = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
hi, lo, val, rep = tab.compact()
b = dv.finalize(hi, lo, val, rep, t, nparts)
def keys(c):
    off = np.asarray(c["key_off"], np.int64); bl = c["key_blob"].tobytes()
    return [bl[off[i]:off[i+1]] for i in range(len(off) - 1)]
ka, kb = keys(a), keys(b)
print("n", len(ka), len(kb), "sorted a?", ka == sorted(ka), "sorted b?", kb == sorted(kb))
bad = [i for i in range(min(len(ka), len(kb))) if ka[i] != kb[i]]
print("mismatches", len(bad))
for i in bad[:10]:
    print(i, ka[i], kb[i], a["val"][i], b["val"][i])
