"""Map kernel on one rank's share of the corpus (1/W of the splits, default
W = 8): cold table (reset before each run: every distinct key is claimed)
against a warm one (keys already present: every flush entry takes the
home-slot fast path), and the tail compaction of that table.
Usage: python tools/map_warm_probe.py [W]"""
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.runtime import device as devmod

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
splits = load_corpus()
share = b"".join(splits[: (len(splits) + W - 1) // W])
dev = torch.frombuffer(bytearray(share), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 20, device="cuda")


def timed(fn, reset):
    ts = []
    for _ in range(9):
        if reset:
            tab.reset()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[0], ts[len(ts) // 2]


print(f"W={W}: {dev.numel() / 1e6:.1f} MB, table cap {tab.cap}")
for name, reset in (("cold", True), ("warm", False)):
    mn, md = timed(lambda: tab.wordcount_map(dev), reset)
    print(f"map {name}: min {mn:.3f} ms med {md:.3f} ms", flush=True)
tab.reset(); tab.wordcount_map(dev)
n, ovf = tab.stats()
print(f"distinct {n}")
for nparts in (10,):
    mn, md = timed(lambda: devmod.compact_partition(tab, n, dev, nparts), False)
    print(f"compact_partition ({n} keys, cap {tab.cap}): min {mn:.3f} ms med {md:.3f} ms", flush=True)
