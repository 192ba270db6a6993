"""Deferred map flush (csrc/hip/wordcount3.hip configs 10-11: entries to
scratch, folded on a side stream while the next piece maps) against the atomic
flush (configs 6, 8) on the full Europarl-shaped corpus in HBM, over piece
counts; min/median ms of one map call and the table check of each.
Usage: python tools/wc_ablate7.py"""
import dataclasses
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import primitives
from lua_mapreduce_1_amd.utils.corpus import europarl_like

text = b"".join(europarl_like())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")
base = primitives.TUNABLES


def run(mode, pieces=8, label=""):
    primitives.TUNABLES = dataclasses.replace(base, wc_pieces=pieces)
    ts = []
    for _ in range(7):
        tab.reset(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev, mode=mode); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    extra = ""
    if mode >> 8 == 0:
        n, ovf = tab.stats()
        hi, lo, val, rep = tab.compact()
        extra = f" distinct={hi.numel()} total={int(val.sum())} overflow={ovf}"
    print(f"{label:28s} min {ts[0]:7.3f} ms med {ts[len(ts)//2]:7.3f} ms{extra}", flush=True)


run(6, label="cfg6 atomic flush")
run(8, label="cfg8 atomic flush")
run(1 << 8 | 6, label="cfg6 no flush")
for c in (10, 11):
    for p in (1, 2, 4, 8, 16, 32):
        run(c, p, label=f"cfg{c} deferred pieces={p}")
run(3 << 8 | 10, 1, label="cfg10 map+scratch, no fold")
run(3 << 8 | 11, 1, label="cfg11 map+scratch, no fold")
primitives.TUNABLES = base
