"""EXPERIMENT A/B: the word-count map kernel with persistent workgroups that
take 4 or 8 tiles each and flush their LDS table after every tile (the next
tile's bytes already in registers while the flush's adds are in flight) vs
the production one-tile workgroups.  Full corpus in HBM, 2^22-slot table,
warm (keys present) and cold (table reset), median of 9; every variant's
table is checked equal to the production one's.
Usage: python tools/map_tiles_ab.py"""
import ctypes
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import _hip

text = b"".join(load_corpus())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
L = _hip.lib()


def table_state(tab):
    hi, lo, val, rep = tab.compact(tab.stats())
    p = ops.sort_keys([hi, lo]).long()
    return hi[p], lo[p], val[p]


ref = None
for k in (1, 4, 8, 1, 4, 8):
    assert L.mr_wc3_set_tiles(ctypes.c_int(k)) == 0
    tab = ops.HashTable(1 << 22, device="cuda")
    res = {}
    for name, reset in (("cold", True), ("warm", False)):
        ts = []
        for _ in range(9):
            if reset:
                tab.reset()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); tab.wordcount_map(dev); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[name] = (ts[0], ts[4])
    tab.reset(); tab.wordcount_map(dev)
    st = table_state(tab)
    if ref is None:
        ref = st
    same = all(torch.equal(a, b) for a, b in zip(st, ref))
    print(f"tiles {k}: cold min {res['cold'][0]:.3f} med {res['cold'][1]:.3f} ms | warm min {res['warm'][0]:.3f} "
          f"med {res['warm'][1]:.3f} ms | distinct {st[0].numel()} equal {same}", flush=True)
    del tab
L.mr_wc3_set_tiles(ctypes.c_int(1))
