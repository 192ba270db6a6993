"""Partitioned map flush (csrc/hip/wordcount3.hip configs 10-12) against the
atomic flush (config 6) on the full Europarl-shaped corpus in HBM: full map,
no flush, the partitioned write without the bucket kernel (ablate 3) and the
bucket kernel alone (ablate 4), min/median ms, and the table check of every
full run.  Usage: python tools/wc_ablate6.py [cfg ...]"""
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

text = b"".join(europarl_like())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")
cfgs = [int(x) for x in sys.argv[1:]] or [6, 10, 11, 12]


def timed(mode, reset=True):
    ts = []
    for _ in range(7):
        if reset:
            tab.reset()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev, mode=mode); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts


for c in cfgs:
    modes = [(0, "full"), (1, "no-flush")] + ([(3, "part-write"), (4, "bucket-only"), (5, "bucket-gather")]
                                              if c >= 10 else [])
    for mode, name in modes:
        if mode >= 4:
            tab.reset(); tab.wordcount_map(dev, mode=(3 << 8) | c)  # scratch of one map launch
        ts = timed((mode << 8) | c, reset=(mode < 4))
        extra = ""
        if mode == 0:
            n, ovf = tab.stats()
            hi, lo, val, rep = tab.compact()
            extra = f" distinct={hi.numel()} total={int(val.sum())} overflow={ovf}"
        print(f"cfg{c} {name:11s} min {ts[0]:7.3f} ms med {ts[len(ts)//2]:7.3f} ms "
              f"{dev.numel() / ts[0] / 1e6:7.1f} GB/s{extra}", flush=True)
