"""Host roctx ranges and GPU kernels of one steady-state iteration on one
time axis (rocprofv3 --marker-trace --kernel-trace of a run with MR_ROCTX=1).

    python tools/host_gpu_timeline.py <dir with run_marker_api_trace.csv and run_kernel_trace.csv> [back=3]
"""
import csv
import os
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
mk = sorted(csv.DictReader(open(os.path.join(d, "run_marker_api_trace.csv"))),
            key=lambda r: int(r["Start_Timestamp"]))
kt = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
its = [r for r in mk if r["Function"] == "mr.iteration"]
a, b = its[-back - 1], its[-back]
t0, t1 = int(a["Start_Timestamp"]), int(b["Start_Timestamp"])
ev = []
for r in mk:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1:
        ev.append((s, e, "HOST", r["Function"]))
for r in kt:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1 or (s < t0 < e):
        ev.append((s, e, "s" + r["Stream_Id"], r["Kernel_Name"].split("(")[0][-56:]))
ev.sort()
print(f"iteration span {(t1 - t0) / 1e3:.1f} us")
for s, e, who, name in ev:
    print(f"{(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f} ({(e - s) / 1e3:6.1f})  {who:5s} {name}")
