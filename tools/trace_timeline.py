#!/usr/bin/env python
"""Compact timeline of a rocprofv3 run (kernel trace + memory-copy trace):
per stream/engine, the busy intervals of the last ``--window-ms`` of the
run merged, with the kernels and copies in them — to see whether copies and
kernels overlap and where the device idles.

    python tools/trace_timeline.py DIR [--window-ms 20] [--merge-us 20]
"""
import argparse
import csv
import glob
import os


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append(("K" + r.get("Queue_Id", "?"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            nb = r.get("Bytes") or r.get("Size") or "?"
            ev.append(("C" + r.get("Direction", r.get("Kind", "?"))[:12], int(r["Start_Timestamp"]),
                       int(r["End_Timestamp"]), f"copy {nb} B"))
    return sorted(ev, key=lambda e: e[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window-ms", type=float, default=20.0)
    ap.add_argument("--merge-us", type=float, default=20.0)
    a = ap.parse_args()
    ev = load(a.dir)
    if not ev:
        print("no events")
        return
    t_end = max(e[2] for e in ev)
    t0 = t_end - int(a.window_ms * 1e6)
    ev = [e for e in ev if e[2] >= t0]
    lanes = sorted({e[0] for e in ev})
    for lane in lanes:
        es = [e for e in ev if e[0] == lane]
        busy = sum(e[2] - e[1] for e in es)
        print(f"== {lane}: {len(es)} events, busy {busy / 1e6:.3f} ms of {a.window_ms} ms")
        seg = None
        for e in es:
            if seg and e[1] - seg[1] <= a.merge_us * 1e3:
                seg[1] = max(seg[1], e[2])
                seg[2][e[3]] = seg[2].get(e[3], 0) + 1
            else:
                if seg:
                    print(f"   {(seg[0] - t0) / 1e6:8.3f} .. {(seg[1] - t0) / 1e6:8.3f} ms  "
                          + ", ".join(f"{k} x{v}" for k, v in list(seg[2].items())[:4]))
                seg = [e[1], e[2], {e[3]: 1}]
        if seg:
            print(f"   {(seg[0] - t0) / 1e6:8.3f} .. {(seg[1] - t0) / 1e6:8.3f} ms  "
                  + ", ".join(f"{k} x{v}" for k, v in list(seg[2].items())[:4]))


if __name__ == "__main__":
    main()
