"""Kernel statistics (the columns of rocprofv3's kernel_stats.csv) from a
rocprofv3 rocpd database (``run_results.db``, ROCm 7's default output format):
``python tools/rocpd_kstats.py run_results.db > kernel_stats.csv``."""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = c.execute("SELECT name, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), "
                     "MAX(end - start) FROM kernels GROUP BY name ORDER BY SUM(end - start) DESC").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 4), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
