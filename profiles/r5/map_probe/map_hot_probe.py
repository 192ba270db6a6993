"""Timing probe: how much of the word-count map kernel is the flush of the
most frequent (short) words?  The full corpus in HBM, a warm table; the
flush of packed keys of at most L bytes is dropped (mr_wc3_probe_skip, counts
wrong) for L = 0 (off), 1, 2, 3, 4; prints the kernel time and the share of
flush entries those keys are (host count over the corpus, per 8 KiB tile).
Usage: python tools/map_hot_probe.py"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import _hip

splits = load_corpus()
data = b"".join(splits)
dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 23, device="cuda")

# flush entries per tile by key length (host): distinct words whose first byte is in an 8 KiB tile
tile = 8192
ent = np.zeros(8, np.int64)
tot = 0
for t0 in range(0, min(len(data), 64 * 2**20), tile):  # the first 64 MB
    words = set(data[t0:t0 + tile].split())
    tot += len(words)
    for w in words:
        if len(w) <= 7:
            ent[len(w)] += 1
print(f"flush entries per tile (first 64 MB): {tot / (min(len(data), 64 * 2**20) / tile):.0f}; "
      f"share of keys of <= L bytes: " + ", ".join(f"L={L}: {ent[1:L + 1].sum() / tot:.2f}" for L in range(1, 8)),
      flush=True)


def timed(fn):
    ts = []
    for _ in range(11):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[0], ts[len(ts) // 2]


tab.wordcount_map(dev)  # warm: every key claimed
for L in (0, 1, 2, 3, 4, 5, 6, 7, 0):
    _hip.lib().mr_wc3_probe_skip(L)
    mn, md = timed(lambda: tab.wordcount_map(dev))
    print(f"skip packed keys <= {L} bytes: map min {mn:.3f} ms med {md:.3f} ms", flush=True)
_hip.lib().mr_wc3_probe_skip(0)
