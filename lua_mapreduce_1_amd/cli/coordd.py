"""Stand-alone coordinator daemon (the mongod of this framework).

    python -m lua_mapreduce_1_amd.cli.coordd [--host 0.0.0.0] [--port 27027] [--journal PATH]

With ``--journal`` every mutating request is appended to PATH and replayed on
restart, so a crashed server can resume a task (server.lua:469-502 restart
semantics) and persistent tables survive.
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="coordd")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=27027)
    ap.add_argument("--journal", default=None)
    a = ap.parse_args(argv)
    from ..runtime import coordinator
    return coordinator.serve_forever(a.port, a.host, a.journal)


if __name__ == "__main__":
    sys.exit(main())
