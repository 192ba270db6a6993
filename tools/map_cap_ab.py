"""Word-count map kernel (config 6) on the full corpus in HBM against the HBM
table's capacity: a smaller table keeps more of its tag array in the XCDs' L2,
so the flush's speculative loads wait less; a fuller one probes longer.  Cold
table per run (reset + map), min / median of 9, plus the warm map (keys
present).  Usage: python tools/map_cap_ab.py [log2cap ...]"""
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops

text = b"".join(load_corpus())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
for lc in [int(x) for x in sys.argv[1:]] or [19, 20, 21, 22]:
    tab = ops.HashTable(1 << lc, device="cuda")
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
        res[name] = (ts[0], ts[len(ts) // 2])
    tab.reset(); tab.wordcount_map(dev)
    n, ovf = tab.stats()
    print(f"cap 2^{lc}: cold min {res['cold'][0]:6.3f} med {res['cold'][1]:6.3f} ms | warm min {res['warm'][0]:6.3f} "
          f"med {res['warm'][1]:6.3f} ms | distinct {n} load {n / tab.cap:.2f} overflow {ovf}", flush=True)
    del tab
