"""Ablation timing of the word-count map kernels (v1 vs v2 modes)."""
import sys, time
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
for name, fn in [
    ("v1 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536, version=1)),
    ("v2 full 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536)),
    ("v2 full 32K", lambda: tab.wordcount_map(dev, chunk_bytes=32768)),
    ("v2 full 16K", lambda: tab.wordcount_map(dev, chunk_bytes=16384)),
    ("v2 full staged 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536, mode=4)),
    ("v2 full staged 32K", lambda: tab.wordcount_map(dev, chunk_bytes=32768, mode=4)),
    ("v2 full staged 16K", lambda: tab.wordcount_map(dev, chunk_bytes=16384, mode=4)),
    ("v2 tokenize-only 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536, mode=1)),
    ("v2 lds-only 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536, mode=2)),
    ("v2 lds+flush 64K", lambda: tab.wordcount_map(dev, chunk_bytes=65536, mode=3)),
]:
    mn, md = timeit(fn)
    extra = ""
    if "full" in name:
        n, ovf = tab.stats(); c = int(tab._ovf_counter.item())
        hi, lo, val, rep = tab.compact(); extra = f"distinct={hi.numel()} total={int(val.sum())} overflow_tokens={c}"
    print(f"{name:24s} min {mn:7.3f} ms  med {md:7.3f} ms  {len(text)/mn/1e6:7.1f} GB/s {extra}", flush=True)
