"""Generic worker launcher (reference: execute_worker.lua).

    python -m lua_mapreduce_1_amd.cli.execute_worker CONN DBNAME [--max-iter N] [--max-sleep S] [--max-tasks T]
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="execute_worker")
    ap.add_argument("connection_string")
    ap.add_argument("dbname")
    ap.add_argument("--max-iter", type=int, default=20)
    ap.add_argument("--max-sleep", type=float, default=20)
    ap.add_argument("--max-tasks", type=int, default=1)
    ap.add_argument("--poll", type=float, default=None)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    from .. import worker
    w = worker.new(a.connection_string, a.dbname)
    cfg = dict(max_iter=a.max_iter, max_sleep=a.max_sleep, max_tasks=a.max_tasks, verbose=not a.quiet)
    if a.poll is not None:
        cfg["poll_sleep"] = a.poll
    w.configure(cfg)
    w.execute()
    return 0


if __name__ == "__main__":
    sys.exit(main())
