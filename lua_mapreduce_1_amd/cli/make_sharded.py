"""Blob-store sharding admin tool (reference: misc/make_sharded.lua, which
enables MongoDB sharding of ``<db>.fs.chunks`` on ``files_id``).

Here the blob store scales out by listing several coordinator endpoints in the
connection string (``"h1:p1,h2:p2,..."``): blobs are placed by FNV-1(file name)
mod #endpoints, the first endpoint keeps the job tables.  This tool checks
that every endpoint answers, reports the per-shard blob counts/bytes of a
database and, with ``--rebalance``, moves every blob to its home shard (needed
after adding an endpoint to a running deployment).

    python -m lua_mapreduce_1_amd.cli.make_sharded h1:p1,h2:p2 dbname [--rebalance]
"""
from __future__ import annotations

import argparse
import sys

from ..runtime.cnn import cnn as cnn_cls, shard_of, split_endpoints


def status(connection_string: str, dbname: str) -> list[dict]:
    g = cnn_cls(connection_string, dbname).gridfs()
    eps = split_endpoints(connection_string)
    out = []
    for i, c in enumerate(g.shards):
        st, _ = c.request("PING", "")
        _, f = c.request("BLOB_LIST", dbname, "")
        names = [f[j].decode("utf-8", "surrogateescape") for j in range(0, len(f), 2)]
        sizes = [int(f[j + 1]) for j in range(0, len(f), 2)]
        misplaced = sum(1 for n in names if shard_of(n, len(g.shards)) != i)
        out.append({"endpoint": eps[i], "alive": st == 0, "blobs": len(names), "bytes": sum(sizes),
                    "misplaced": misplaced})
    return out


def rebalance(connection_string: str, dbname: str) -> int:
    """Move every blob to its home shard; returns the number moved."""
    g = cnn_cls(connection_string, dbname).gridfs()
    moved = 0
    n = len(g.shards)
    for i, c in enumerate(g.shards):
        _, f = c.request("BLOB_LIST", dbname, "")
        for j in range(0, len(f), 2):
            name = f[j].decode("utf-8", "surrogateescape")
            home = shard_of(name, n)
            if home == i:
                continue
            st, data = c.request("BLOB_GET", dbname, name)
            if st != 0:
                continue
            g.shards[home].request("BLOB_PUT", dbname, name, data[0])
            c.request("BLOB_DEL", dbname, name)
            moved += 1
    return moved


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("connection_string")
    ap.add_argument("dbname")
    ap.add_argument("--rebalance", action="store_true")
    a = ap.parse_args(argv)
    if a.rebalance:
        print("# moved %d blobs" % rebalance(a.connection_string, a.dbname))
    rows = status(a.connection_string, a.dbname)
    for r in rows:
        print("%-24s alive=%-5s blobs=%-8d bytes=%-12d misplaced=%d" % (r["endpoint"], r["alive"], r["blobs"],
                                                                     r["bytes"], r["misplaced"]))
    return 0 if all(r["alive"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
