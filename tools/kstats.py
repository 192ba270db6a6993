#!/usr/bin/env python
"""Print the top kernels of a rocprofv3 kernel_stats.csv (ms total, calls,
average us, share) — python tools/kstats.py FILE [TOP]."""
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    for r in rows[:top]:
        print(f'{float(r["TotalDurationNs"]) / 1e6:9.2f} ms {int(r["Calls"]):6d} x {float(r["AverageNs"]) / 1e3:9.1f} us '
              f'{float(r["Percentage"]):5.1f}%  {r["Name"][:110]}')


if __name__ == "__main__":
    main()
