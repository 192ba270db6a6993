"""One iteration of tools/proxy_terasort.py from a rocprofv3 kernel trace:
the kernels between the last two full-block key passes (rec_keys32 over the
rank's whole block; the last one is the proxy's own check after timing), with
their stream, start and duration, and per-stream busy time — shows how far
the exchange rounds (the model's copy + hold on its own stream) overlap the
receive-side sorts.

    python tools/proxy_timeline.py kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


keys = [i for i, r in enumerate(rows) if "keys32" in r["Kernel_Name"]]
big = max(dur(rows[i]) for i in keys)
full = [i for i in keys if dur(rows[i]) > big // 2]
a, b = full[-2], full[-1]
t0 = int(rows[a]["Start_Timestamp"])
busy = defaultdict(int)
end = t0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[r["Stream_Id"]] += e - s
    end = max(end, e)
    print(f"{(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us  s{r['Stream_Id']:>3}  {r['Kernel_Name'].split('(')[0][-64:]}")
print(f"window {(end - t0) / 1e3:.1f} us; busy per stream: "
      + ", ".join(f"s{k} {v / 1e3:.1f} us" for k, v in sorted(busy.items())))
