"""Word-count map kernel: v2 (16 KiB) vs the v3 configurations (occupancy /
prefetch ablation), full Europarl-shaped corpus in HBM, one launch each."""
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

splits = europarl_like()
text = b"".join(splits)
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
sub = dev[: len(text) // 8]  # one rank's share at 8 GPUs
tab = ops.HashTable(1 << 21, device="cuda")
def timeit(fn, reps=5):
    ts = []
    for _ in range(reps):
        tab.reset(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts), sorted(ts)[len(ts)//2]
cfgs = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3, 4, 5]
for data, tag in ((dev, "full"), (sub, "1/8 ")):
    runs = []
    runs += [(f"v3 cfg{c}", (lambda c=c: tab.wordcount_map(data, mode=c))) for c in cfgs]
    for name, fn in runs:
        mn, md = timeit(fn)
        n, ovf = tab.stats(); cnt = int(tab._ovf_counter.item())
        hi, lo, val, rep = tab.compact()
        print(f"{tag} {name:8s} min {mn:7.3f} ms med {md:7.3f} ms {data.numel()/mn/1e6:7.1f} GB/s "
              f"distinct={hi.numel()} total={int(val.sum())} ovf_tokens={cnt} overflow={ovf}", flush=True)
# warm table: the same 1/8 input again without a reset (every key already
# present: no claims) — isolates the cost of new-key claims
for c in cfgs[:3]:
    ts = []
    for _ in range(5):
        tab.reset(); tab.wordcount_map(sub, mode=c); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(sub, mode=c); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"1/8 warm-table v3 cfg{c} min {min(ts):7.3f} ms", flush=True)
