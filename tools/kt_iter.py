"""Print the kernel sequence of the last iterations of a rocprofv3 kernel trace,
anchored on one kernel name that runs once per iteration."""
import csv, sys
path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "table_reset"
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
print(len(rows), "kernels,", len(starts), "anchors")
for k in range(max(0, len(starts) - 1 - nshow), len(starts) - 1):
    a, b = starts[k], starts[k + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev = None
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        gap = (s - prev) / 1e3 if prev else 0
        print(f"{(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {r['Kernel_Name'][:60]}")
        prev = e
    print(f"---- span {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
