#!/usr/bin/env python
"""Kernels and memory copies of one steady iteration on one time axis, from a
``rocprofv3 --kernel-trace --memory-copy-trace`` directory.  Iterations are
cut at the first launch of ``--anchor`` (a kernel name substring) after a gap
of more than ``--gap-ms`` since its previous launch; the listing covers the
``--back``-th iteration from the end and ends with per-stream busy time.

    python tools/copy_kernel_timeline.py DIR [--anchor agg_combine] [--back 2] [--min-us 50]
"""
import argparse
import collections
import csv
import glob
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--anchor", default="agg_combine")
    ap.add_argument("--gap-ms", type=float, default=5.0)
    ap.add_argument("--back", type=int, default=2)
    ap.add_argument("--min-us", type=float, default=50.0)
    a = ap.parse_args()
    kt = sorted(csv.DictReader(open(glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))[0])),
                key=lambda r: int(r["Start_Timestamp"]))
    cps = glob.glob(os.path.join(a.dir, "*memory_copy_trace.csv"))
    ct = sorted(csv.DictReader(open(cps[0])), key=lambda r: int(r["Start_Timestamp"])) if cps else []
    anchors = [int(r["Start_Timestamp"]) for r in kt if a.anchor in r["Kernel_Name"]]
    starts = [t for i, t in enumerate(anchors) if i == 0 or t - anchors[i - 1] > a.gap_ms * 1e6]
    t0, t1 = starts[-a.back - 1], starts[-a.back]
    ev = []
    busy = collections.Counter()
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            who = "k" + r.get("Stream_Id", r.get("Queue_Id", "?"))
            busy[who] += e - s
            ev.append((s, e, who, r["Kernel_Name"].split("(")[0][-60:]))
    for r in ct:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
            size = r.get("Size") or r.get("Bytes") or "?"
            busy["copy " + kind] += e - s
            ev.append((s, e, "copy", f"{kind} {size} B"))
    print(f"iteration span {(t1 - t0) / 1e6:.3f} ms")
    for s, e, who, name in sorted(ev):
        if (e - s) / 1e3 >= a.min_us:
            print(f"{(s - t0) / 1e3:9.1f} -> {(e - t0) / 1e3:9.1f} ({(e - s) / 1e3:8.1f} us)  {who:8s} {name}")
    print("busy per stream / copy kind (ms):")
    for k, v in busy.most_common():
        print(f"  {k:30s} {v / 1e6:8.3f}")


if __name__ == "__main__":
    main()
