"""Kernel-level timing of the word-count map path on one GPU (dev tool)."""
import sys, time
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

t0 = time.time()
splits = europarl_like()
text = b"".join(splits)
print(f"corpus {len(text)/1e6:.1f} MB gen {time.time()-t0:.1f}s", flush=True)
host = torch.frombuffer(bytearray(text), dtype=torch.uint8).pin_memory()
dev = host.cuda()
for chunk in (32 * 1024, 64 * 1024, 128 * 1024, 256 * 1024):
    tab = ops.HashTable(1 << 21, device="cuda")
    for it in range(3):
        tab.reset()
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        tab.wordcount_map(dev, chunk_bytes=chunk)
        e1.record()
        hi, lo, val, rep = tab.compact()
        e2.record()
        torch.cuda.synchronize()
    print(f"chunk {chunk//1024}K: map {e0.elapsed_time(e1):.3f} ms  compact {e1.elapsed_time(e2):.3f} ms "
          f"distinct {hi.numel()} total {int(val.sum())}", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); dev2 = host.to("cuda", non_blocking=True); e1.record(); torch.cuda.synchronize()
print(f"H2D {len(text)/1e6:.0f} MB: {e0.elapsed_time(e1):.3f} ms", flush=True)
p = ops.sort_keys([hi, lo]); torch.cuda.synchronize()
e0.record(); p = ops.sort_keys([hi, lo]); e1.record(); torch.cuda.synchronize()
print(f"sort {hi.numel()} keys (128-bit): {e0.elapsed_time(e1):.3f} ms", flush=True)
