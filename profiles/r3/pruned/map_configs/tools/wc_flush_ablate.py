"""Where the map kernel's flush time goes (config 6, full corpus in HBM, warm
table: every key already claimed, as in the steady state of a corpus that
repeats): full flush, home-slot tag load only (no lo/hi loads: what a slot
layout with tag, hi, lo in one line would load), blind atomic adds (no
loads), loads only (no atomics), no flush.  Timing only (ablations leave the
table wrong).  Usage: python tools/wc_flush_ablate.py [cfg]"""
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 6
text = b"".join(load_corpus())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")
for mode, name in ((0, "full flush (cold table)"), (0, "full flush (warm table)"), (3, "tag load only"),
                   (4, "blind atomics"), (5, "loads only"), (1, "no flush")):
    ts = []
    for _ in range(9):
        tab.reset()
        if "cold" not in name:
            tab.wordcount_map(dev, mode=cfg)  # warm: every key claimed
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev, mode=(mode << 8) | cfg); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(f"cfg{cfg} {name:24s} min {ts[0]:7.3f} ms med {ts[len(ts) // 2]:7.3f} ms", flush=True)
