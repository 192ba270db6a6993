"""Ablation of the word-count map kernel at small chunks: where the time goes
(tokenize / LDS combine / flush to the HBM table / overflow)."""
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

splits = europarl_like()
text = b"".join(splits)
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")
def timeit(fn, reps=5):
    ts = []
    for _ in range(reps):
        tab.reset(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts), sorted(ts)[len(ts)//2]
modes = [(m, c) for c in (8192, 16384, 32768) for m in (0, 1, 2, 3)]
extra_modes = [int(x) for x in sys.argv[1:]]
modes += [(m, c) for m in extra_modes for c in (8192, 16384, 32768, 65536)]
names = {0: "full", 1: "tokenize", 2: "lds-only", 3: "lds+flush", 4: "staged", 5: "m5", 6: "m6", 7: "m7"}
for m, c in modes:
    mn, md = timeit(lambda: tab.wordcount_map(dev, chunk_bytes=c, mode=m))
    extra = ""
    if m in (0, 4) or m >= 5:
        n, ovf = tab.stats(); cnt = int(tab._ovf_counter.item())
        hi, lo, val, rep = tab.compact()
        extra = f"distinct={hi.numel()} total={int(val.sum())} ovf_tokens={cnt} overflow={ovf}"
    print(f"{names.get(m, m):10s} {c//1024:3d}K min {mn:7.3f} ms med {md:7.3f} ms {len(text)/mn/1e6:7.1f} GB/s {extra}",
          flush=True)
