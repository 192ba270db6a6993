"""EXPERIMENT (timing only, results invalid when spread != 0): the word-count
map kernel with the flush's fast-path atomic adds spread over 8 addresses per
key (by workgroup), to test whether same-address serialisation of the hot
words' adds at the memory side bounds the flush.  Warm table (keys present),
median of 9.  Usage: python tools/map_spread_probe.py"""
import ctypes
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import _hip

text = b"".join(load_corpus())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 22, device="cuda")
tab.wordcount_map(dev)
for spread in (0, 1 << 19, 0, 1 << 19, 1 << 12):
    _hip.lib().mr_wc3_set_spread(ctypes.c_ulonglong(spread))
    ts = []
    for _ in range(9):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(f"spread {spread:8d}: warm min {ts[0]:.3f} med {ts[4]:.3f} ms", flush=True)
_hip.lib().mr_wc3_set_spread(ctypes.c_ulonglong(0))
