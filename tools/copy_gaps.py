#!/usr/bin/env python
"""Copy-engine occupancy of a steady run, from a ``rocprofv3 --kernel-trace
--memory-copy-trace`` directory: host->device bytes, the time the H2D copies
were busy against the wall time of the window, and the largest gaps between
consecutive H2D copies with the kernels that ran inside each gap.

A pipeline bound by its input copies keeps the copy engine busy; gaps mean
the host issued the next copies late (it was waiting on the device).

    python tools/copy_gaps.py DIR [--skip-ms 200] [--top 12]
"""
import argparse
import csv
import glob
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip-ms", type=float, default=0.0, help="ignore the first ms of copies (warm-up)")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--min-bytes", type=int, default=1 << 20, help="H2D copies at least this large")
    a = ap.parse_args()
    kt = sorted(csv.DictReader(open(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0])),
                key=lambda r: int(r["Start_Timestamp"]))
    ct = sorted(csv.DictReader(open(glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"),
                                              recursive=True)[0])), key=lambda r: int(r["Start_Timestamp"]))
    h2d = [r for r in ct if "HOST_TO_DEVICE" in r.get("Direction", "") and int(r.get("Size", 0)) >= a.min_bytes]
    if not h2d:
        print("no H2D copies")
        return
    t0 = int(h2d[0]["Start_Timestamp"]) + int(a.skip_ms * 1e6)
    h2d = [r for r in h2d if int(r["Start_Timestamp"]) >= t0]
    start, end = int(h2d[0]["Start_Timestamp"]), int(h2d[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in h2d)
    nbytes = sum(int(r["Size"]) for r in h2d)
    wall = end - start
    print(f"H2D copies {len(h2d)}, {nbytes / 1e9:.3f} GB in {wall / 1e6:.3f} ms wall; busy {busy / 1e6:.3f} ms "
          f"({100.0 * busy / max(wall, 1):.1f}%); {nbytes / max(busy, 1):.1f} GB/s while busy, "
          f"{nbytes / max(wall, 1):.1f} GB/s overall")
    gaps = []
    for p, q in zip(h2d, h2d[1:]):
        g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
        if g > 0:
            gaps.append((g, int(p["End_Timestamp"]), int(q["Start_Timestamp"])))
    tot = sum(g for g, _, _ in gaps)
    print(f"gaps: {len(gaps)}, total {tot / 1e6:.3f} ms")
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]) for r in kt]
    for g, a0, b0 in sorted(gaps, reverse=True)[:a.top]:
        inside = [k for k in ks if k[1] > a0 and k[0] < b0]
        names = {}
        for s, e, n in inside:
            names[n] = names.get(n, 0) + (min(e, b0) - max(s, a0))
        top = sorted(names.items(), key=lambda x: -x[1])[:4]
        print(f"  gap {g / 1e3:8.1f} us at +{(a0 - start) / 1e6:9.3f} ms; kernels busy inside: " +
              ", ".join(f"{n} {v / 1e3:.0f}us" for n, v in top))


if __name__ == "__main__":
    main()
