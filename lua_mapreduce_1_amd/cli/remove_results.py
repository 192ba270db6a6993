"""Drop every collection / blob of a database (reference: remove_results.sh).

    python -m lua_mapreduce_1_amd.cli.remove_results CONN DBNAME
"""
from __future__ import annotations

import sys


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        print(__doc__)
        return 2
    from ..runtime.coordinator import Client
    Client(argv[0]).request("DB_DROP", argv[1])
    return 0


if __name__ == "__main__":
    sys.exit(main())
