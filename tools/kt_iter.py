"""Print one iteration of a rocprofv3 kernel trace: from a table reset that
is followed by a map launch to the next such reset (second to last by default)."""
import csv
import sys

path = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "table_reset" in r["Kernel_Name"]
       and any("map" in rows[j]["Kernel_Name"] for j in range(i + 1, min(i + 4, len(rows))))]
a, b = idx[-back - 1], idx[-back]
t0 = int(rows[a]["Start_Timestamp"])
prev, busy = None, 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us gap {gap:6.1f}  {r['Kernel_Name'][:58]}")
    prev = e
print(f"span {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
