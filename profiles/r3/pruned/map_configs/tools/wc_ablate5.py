"""Map kernel configurations x phase ablation (full / no flush / tokenize only)
on the full Europarl-shaped corpus in HBM: v3 configs 0-5 and the dense
token-list configs 6-9 (csrc/hip/wordcount3.hip).  Prints min/median ms and the
table check (distinct keys, total count) of every full run."""
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

text = b"".join(europarl_like())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
# MR_ABLATE_LOG2CAP: table capacity (default 2^21; the engine uses 2^22 for the full corpus, sparse tables)
import os
tab = ops.HashTable(1 << int(os.environ.get("MR_ABLATE_LOG2CAP", "21")), device="cuda")
cfgs = [int(x) for x in sys.argv[1:]] or [0, 6, 1, 7, 3, 8, 2, 9]
for c in cfgs:
    for mode, name in ((0, "full"), (1, "no-flush"), (2, "tokenize")):
        ts = []
        for _ in range(7):
            tab.reset(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); tab.wordcount_map(dev, mode=(mode << 8) | c); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        extra = ""
        if mode == 0:
            n, ovf = tab.stats()
            hi, lo, val, rep = tab.compact()
            extra = f" distinct={hi.numel()} total={int(val.sum())} overflow={ovf}"
        ts.sort()
        print(f"cfg{c} {name:9s} min {ts[0]:7.3f} ms med {ts[len(ts)//2]:7.3f} ms "
              f"{dev.numel() / ts[0] / 1e6:7.1f} GB/s{extra}", flush=True)
