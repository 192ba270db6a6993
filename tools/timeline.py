"""Summarise a rocprofv3 kernel trace: per-iteration span, busy time by kernel, idle gaps."""
import csv, sys, collections
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "table_compact" in r["Kernel_Name"]]
# iteration k spans from the row after compact k-1's iteration tail to compact k's tail: use compact as anchor
for k in range(1, len(marks)):
    a, b = marks[k - 1] + 1, marks[k] + 1
    # extend b to include the post-compact tail (until the next big gap > 500us)
    while b < len(rows) and int(rows[b]["Start_Timestamp"]) - int(rows[b - 1]["End_Timestamp"]) < 500_000 \
            and "wc_map" not in rows[b]["Kernel_Name"]:
        b += 1
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = collections.Counter()
    for r in seg:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        busy[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    gaps = sorted(((int(seg[i]["Start_Timestamp"]) - int(seg[i - 1]["End_Timestamp"]), seg[i]["Kernel_Name"][:40])
                   for i in range(1, len(seg))), reverse=True)[:4]
    print(f"iter {k}: span {(t1 - t0) / 1e6:.3f} ms, busy {sum(busy.values()) / 1e6:.3f} ms, launches {len(seg)}")
    for n, v in busy.most_common(6):
        print(f"    {v / 1e6:7.3f} ms  {n}")
    print("    largest gaps (us):", [(round(g / 1e3, 1), n) for g, n in gaps])
