#!/usr/bin/env python
"""Per-dispatch medians of rocprofv3 --pmc counter CSVs (one directory per
pass): counters summed over a dispatch's rows, then the median over the
dispatches of the selected kernel.

    python tools/pmc_summary.py DIR [DIR ...] [--kernel REGEX]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re
import statistics


def summarize(d: str, kernel: str) -> dict:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(kernel, r["Kernel_Name"]):
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}
    names = sorted({n for v in per.values() for n in v})
    out = {n: statistics.median(v[n] for v in per.values() if n in v) for n in names}
    out["_dispatches"] = len(per)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default=".")
    a = ap.parse_args()
    for d in a.dirs:
        for k, v in summarize(d, a.kernel).items():
            print(f"{os.path.basename(d.rstrip('/'))}\t{k}\t{v:.6g}")


if __name__ == "__main__":
    main()
