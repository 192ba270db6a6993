"""Unit-test aggregator (reference: mapreduce/test.lua:19-41): run every
module's ``utest`` in the reference's order and print ``Ok``.

    python -m lua_mapreduce_1_amd.test [connection_string]

Without a connection string an in-process coordinator is used.
"""
from __future__ import annotations

import sys


def run(connection_string=None) -> None:
    from . import utils
    from .runtime import cnn, fs, job, persistent_table, server, task, worker
    import importlib
    # the package attributes ``utils.heap`` / ``utils.tuple`` are the class and
    # the factory; the modules hold the utests
    heap = importlib.import_module(".utils.heap", __package__)
    tuple_mod = importlib.import_module(".utils.tuple", __package__)
    if connection_string is None:
        from .runtime import coordinator
        connection_string = coordinator.start_local()
    utils.utest(connection_string)
    cnn.utest(connection_string)
    fs.utest(connection_string)
    job.utest()
    task.utest()
    server.utest(connection_string)
    worker.utest()
    persistent_table.utest(connection_string)
    heap.utest()
    tuple_mod.utest()


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    run(argv[0] if argv else None)
    print("Ok")
    return 0


if __name__ == "__main__":
    sys.exit(main())
