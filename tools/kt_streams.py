"""Steady-state view of a rocprofv3 kernel trace with two or more streams:
per-iteration span, union-busy time (any kernel running), per-stream busy,
and the kernels of one iteration with their stream — shows whether the GPU or
the host (gaps with nothing running) sets the step time.

    python tools/kt_streams.py run_kernel_trace.csv [iterations=8]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
nit = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
maps = [i for i, r in enumerate(rows) if "map3_kernel" in r["Kernel_Name"] or "wc_map" in r["Kernel_Name"]]
# steady state: between the map launches of the last nit+2 iterations (skip the last two)
sel = maps[-(nit + 2):-1]
a, b = sel[0], sel[-1]
t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
win = [r for r in rows[a:b]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
union, cs, ce = 0, None, None
for s, e in iv:
    if ce is None or s > ce:
        if ce is not None:
            union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
per_stream = defaultdict(int)
per_kernel = defaultdict(lambda: [0, 0])
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per_stream[r["Stream_Id"]] += d
    k = r["Kernel_Name"].split("(")[0][-60:]
    per_kernel[k][0] += d
    per_kernel[k][1] += 1
n = len(sel) - 1
span = (t1 - t0) / 1e3 / n
print(f"{n} iterations: {span:.1f} us/iteration, union-busy {union / 1e3 / n:.1f} us "
      f"({100 * union / (t1 - t0):.0f}%), idle {(t1 - t0 - union) / 1e3 / n:.1f} us")
for s, v in sorted(per_stream.items()):
    print(f"  stream {s}: busy {v / 1e3 / n:.1f} us/iteration")
print("per-iteration kernel time:")
for k, (d, c) in sorted(per_kernel.items(), key=lambda x: -x[1][0]):
    print(f"  {d / 1e3 / n:8.1f} us  x{c / n:4.1f}  {k}")
print("one iteration (start, duration, stream):")
a2, b2 = sel[-2], sel[-1]
tb = int(rows[a2]["Start_Timestamp"])
for r in rows[a2:b2]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {(s - tb) / 1e3:8.1f} +{(e - s) / 1e3:7.1f}  s{r['Stream_Id']}  {r['Kernel_Name'].split('(')[0][-60:]}")
