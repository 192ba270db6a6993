"""Generic server launcher (reference: execute_server.lua).

    python -m lua_mapreduce_1_amd.cli.execute_server CONN DBNAME TASKFN MAPFN PARTITIONFN REDUCEFN \
        [FINALFN] [COMBINERFN|nil] [STORAGE|nil] [INIT_ARGS...]

Module names accept ``/`` or ``.`` separators and an optional ``.py``/``.lua``
suffix.  ``CONN`` is ``host:port`` of a coordinator; when nothing listens
there and the host is local, the server hosts the coordinator itself (the
rank-0 service of SURVEY.md §2.6) so workers can connect to the same address.
Options (before the positionals): ``--device {auto,host}``, ``--sleep S``
(delay before loop, reference: 4 s), ``--journal PATH``.
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="execute_server")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--sleep", type=float, default=4.0)
    ap.add_argument("--journal", default=None)
    ap.add_argument("--poll", type=float, default=None)
    ap.add_argument("connection_string")
    ap.add_argument("dbname")
    ap.add_argument("taskfn")
    ap.add_argument("mapfn")
    ap.add_argument("partitionfn")
    ap.add_argument("reducefn")
    ap.add_argument("rest", nargs="*")
    a = ap.parse_args(argv)
    rest = list(a.rest)
    finalfn = rest.pop(0) if rest else None
    combinerfn = rest.pop(0) if rest else None
    storage = rest.pop(0) if rest else None
    if combinerfn == "nil":
        combinerfn = None
    if storage == "nil":
        storage = None
    if finalfn == "nil":
        finalfn = None
    try:
        sys.stdout.reconfigure(errors="surrogateescape")
    except AttributeError:
        pass
    from .. import server, utils
    from ..runtime import coordinator, modules
    conn = ensure_coordinator(a.connection_string, a.journal)
    s = server.new(conn, a.dbname)
    if a.poll is not None:
        s.poll_sleep = a.poll
    n = modules.normalize
    s.configure({
        "taskfn": n(a.taskfn), "mapfn": n(a.mapfn), "partitionfn": n(a.partitionfn), "reducefn": n(a.reducefn),
        "finalfn": n(finalfn) if finalfn else None, "combinerfn": n(combinerfn) if combinerfn else None,
        "init_args": rest, "storage": storage, "device": a.device,
    })
    utils.sleep(a.sleep)
    s.loop()
    return 0


def ensure_coordinator(cs: str, journal: str | None = None) -> str:
    """Connect to the coordinator at ``cs``; start one in-process when the
    address is local and free."""
    from ..runtime import coordinator
    addr = coordinator.resolve(cs)
    try:
        coordinator.Client(addr, timeout=2.0).ping()
        return addr
    except OSError:
        host, port = addr.rsplit(":", 1)
        if host not in ("127.0.0.1", "localhost", "0.0.0.0"):
            raise
        return coordinator.start_local(int(port), "127.0.0.1" if host != "0.0.0.0" else "0.0.0.0", journal)


if __name__ == "__main__":
    sys.exit(main())
