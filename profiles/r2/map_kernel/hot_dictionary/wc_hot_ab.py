"""Hot-dictionary persistent map (wordcount3.hip mr_wc_map_hot) against the
plain config-6 map on the full Europarl-shaped corpus in HBM: min / median of
9 runs on a cold table each, identical tables checked (distinct keys, every
count); phase ablations of both (no flush / tokenize only), the persistent
map without hot words, and how many tokens the hot counters took.
Usage: python tools/wc_hot_ab.py [grid ...]"""
import dataclasses
import sys
import torch
sys.path.insert(0, ".")
from bench import load_corpus
from lua_mapreduce_1_amd import ops

P = ops.primitives
HOT = P.WC_HOT
# scratch layout (u64 words) of mr_wc_map_hot: wordcount3.hip HS_*
HS_CNT, HS_N = 361490, 372242

text = b"".join(load_corpus())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")


def run(mode, check=True):
    ts = []
    for _ in range(9):
        tab.reset(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); tab.wordcount_map(dev, mode=mode); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    if not check:
        return ts[0], ts[len(ts) // 2], None, None, None
    n, ovf = tab.stats()
    hi, lo, val, rep = tab.compact()
    order = torch.argsort(hi * 1_000_003 + lo)
    return ts[0], ts[len(ts) // 2], n, ovf, (hi[order].cpu(), lo[order].cpu(), val[order].cpu())


mn, md, n, ovf, ref = run(6)
print(f"plain cfg6   min {mn:7.3f} ms med {md:7.3f} ms distinct={n} total={int(ref[2].sum())} overflow={ovf}",
      flush=True)
for name, m in (("no-flush", 1), ("tokenize", 2), ("tag-load", 3), ("blind-atom", 4), ("loads-only", 5)):
    mn, md, *_ = run((m << 8) | 6, check=False)
    print(f"plain cfg6 {name:9s} min {mn:7.3f} ms med {md:7.3f} ms", flush=True)
for grid in [int(x) for x in sys.argv[1:]] or [512]:
    P.TUNABLES = dataclasses.replace(P.TUNABLES, wc_hot_grid=grid)
    mn, md, n, ovf, got = run(HOT)
    same = all(torch.equal(a, b) for a, b in zip(ref, got))
    s = tab._hot_scratch()
    nh = int(s[HS_N]); hot_tokens = int(s[HS_CNT:HS_CNT + 3584].sum())
    print(f"hot grid {grid:4d} min {mn:7.3f} ms med {md:7.3f} ms distinct={n} total={int(got[2].sum())} "
          f"overflow={ovf} identical={same} hot_words={nh} hot_tokens={hot_tokens}", flush=True)
    for name, f in (("no hot words", 1), ("no-flush", 1 << 8), ("tokenize", 2 << 8), ("tag-load", 3 << 8),
                    ("blind-atom", 4 << 8), ("loads-only", 5 << 8), ("hot+blind", 6 << 8),
                    ("nohot+blind", 1 | (6 << 8))):
        mn, md, *_ = run(HOT | (f << 8), check=False)
        print(f"hot grid {grid:4d} {name:12s} min {mn:7.3f} ms med {md:7.3f} ms", flush=True)
