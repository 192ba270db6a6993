import sys, os
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import _hip
splits = load_corpus()
data = b"".join(splits)
dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
ref = None
for tpc in (1, 2, 4, 8, 1):
    _hip.lib().mr_wc3_set_tpc(tpc)
    tab = ops.HashTable(1 << 23, device="cuda")
    ts = []
    for it in range(11):
        if it == 0:
            tab.reset()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    cold = ts[0]; warm = sorted(ts[1:])
    tab.reset(); tab.wordcount_map(dev); torch.cuda.synchronize()
    n, ovf = tab.stats()
    total = int(tab.val.sum()) if hasattr(tab, "val") else -1
    print(f"tpc={tpc}: cold {cold:.3f} ms warm min {warm[0]:.3f} med {warm[len(warm)//2]:.3f} ms distinct {n} total {total} ovf {ovf}", flush=True)
