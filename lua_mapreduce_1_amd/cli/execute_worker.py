"""Generic worker launcher (reference: execute_worker.lua).

    python -m lua_mapreduce_1_amd.cli.execute_worker CONN DBNAME [--max-iter N] [--max-sleep S] [--max-tasks T]
"""
from __future__ import annotations

import argparse
import os
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
    ap.add_argument("--gpu", default="auto", help="auto (one GPU per worker on a multi-GPU node), an index, or none")
    a = ap.parse_args(argv)
    from .. import worker
    prof_dir = os.environ.get("MR_WORKER_PROFILE")
    if prof_dir:  # diagnosis: cProfile of the whole worker, written when it is stopped
        import cProfile
        import pstats
        import signal
        prof = cProfile.Profile()

        def _dump(*_):
            prof.disable()
            os.makedirs(prof_dir, exist_ok=True)
            with open(os.path.join(prof_dir, f"worker_{os.getpid()}.txt"), "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(60)
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
            os._exit(0)
        signal.signal(signal.SIGTERM, _dump)
        prof_dir = os.path.abspath(prof_dir)
        prof.enable()
    else:
        import signal

        def _term(*_):
            raise SystemExit(143)  # unwind: the worker frees its hbm arena (/dev/shm chunks on a CPU node)
        signal.signal(signal.SIGTERM, _term)
    w = worker.new(a.connection_string, a.dbname)
    cfg = dict(max_iter=a.max_iter, max_sleep=a.max_sleep, max_tasks=a.max_tasks, verbose=not a.quiet,
               gpu=a.gpu if a.gpu in ("auto", "none") else int(a.gpu))
    if a.poll is not None:
        cfg["poll_sleep"] = a.poll
    w.configure(cfg)
    w.execute()
    if prof_dir:
        _dump()
    return 0


if __name__ == "__main__":
    sys.exit(main())
