"""Connection layer to the coordinator (reference: mapreduce/cnn.lua).

``cnn(connection_string, dbname, auth_table)`` exposes the same surface as the
reference: ``connect``, ``gridfs`` (blob store), ``grid_file_builder``,
``get_dbname``, the error channel (``insert_error``/``get_errors``/
``remove_errors``) and batched inserts (``annotate_insert`` /
``flush_pending_inserts`` with per-document callbacks, flushed at
``MAX_PENDING_INSERTS``).
"""
from __future__ import annotations

import json
import re
from typing import Callable, Iterator

from .. import utils
from .coordinator import Client, decode_jobs


def split_endpoints(connection_string: str | None) -> list:
    """``"h1:p1,h2:p2,..."`` -> endpoints; the first is the primary (job
    tables, task, errors, persistent tables), all of them hold blobs."""
    if not connection_string or "," not in str(connection_string):
        return [connection_string]
    return [e.strip() for e in str(connection_string).split(",") if e.strip()]


def shard_of(filename: str, nshards: int) -> int:
    """Home shard of a blob: exact uint32 FNV-1 of the name mod nshards."""
    h = 2166136261
    for b in filename.encode("utf-8", "surrogateescape"):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ b
    return h % nshards


class GridFS:
    """Blob store in the coordinator(s) (the GridFS replacement).

    With several coordinator endpoints the blobs are hash-partitioned by file
    name over all of them (the horizontal scale-out the reference gets from
    sharding ``fs.chunks``, misc/make_sharded.lua:69-72); ``list`` merges the
    shards.
    """

    def __init__(self, client, dbname: str):
        self.shards = list(client) if isinstance(client, (list, tuple)) else [client]
        self.c = self.shards[0]
        self.db = dbname

    def _home(self, filename: str):
        return self.shards[shard_of(filename, len(self.shards))] if len(self.shards) > 1 else self.c

    def store_data(self, data: bytes, filename: str) -> bool:
        self._home(filename).request("BLOB_PUT", self.db, filename, bytes(data))
        return True

    def get(self, filename: str) -> bytes | None:
        st, f = self._home(filename).request("BLOB_GET", self.db, filename)
        return f[0] if st == 0 else None

    find_file = get

    # -- batched forms: one round trip per shard (a map job's 15 partition
    # files + their index entries, a reduce job's 197 inputs)
    def _by_shard(self, names):
        groups: dict = {}
        for i, n in enumerate(names):
            c = self._home(n)
            groups.setdefault(id(c), (c, []))[1].append(i)
        return groups.values()

    def store_many(self, items: list[tuple[str, bytes]]) -> None:
        for c, idx in self._by_shard([n for n, _ in items]):
            c.request("BLOB_PUT_MANY", self.db, *[x for i in idx for x in (items[i][0], bytes(items[i][1]))])

    def get_many(self, names: list[str]) -> list[bytes | None]:
        out: list = [None] * len(names)
        for c, idx in self._by_shard(names):
            _, f = c.request("BLOB_GET_MANY", self.db, *[names[i] for i in idx])
            for j, i in enumerate(idx):
                out[i] = f[2 * j + 1] if int(f[2 * j]) else None
        return out

    def remove_many(self, names: list[str]) -> int:
        n = 0
        for c, idx in self._by_shard(names):
            _, f = c.request("BLOB_DEL_MANY", self.db, *[names[i] for i in idx])
            n += int(f[0])
        return n

    def list(self, match: dict | str | None = None, prefix: str = "") -> list[dict]:
        """Files whose name matches a regex (``{"filename": {"$regex": r}}``
        or a plain regex string); all files when ``match`` is None.
        ``prefix``: a literal prefix every match has (filtered by the
        coordinator: the whole store is not sent over)."""
        rx = _regex_of(match)
        out = []
        for c in self.shards:
            _, f = c.request("BLOB_LIST", self.db, prefix)
            names = [(f[i].decode("utf-8", "surrogateescape"), int(f[i + 1])) for i in range(0, len(f), 2)]
            out += [{"filename": n, "length": sz} for n, sz in names if rx is None or rx.search(n)]
        return out

    def remove_file(self, filename: str) -> bool:
        _, f = self._home(filename).request("BLOB_DEL", self.db, filename)
        return int(f[0]) > 0

    def lines(self, filename: str) -> Iterator[bytes]:
        data = self.get(filename) or b""
        for line in data.split(b"\n"):
            if line:
                yield line


def _regex_of(match):
    if match is None:
        return None
    if isinstance(match, dict):
        match = match["filename"]["$regex"]
    return re.compile(match)


class GridFileBuilder:
    def __init__(self, gridfs: GridFS):
        self.fs = gridfs
        self.parts: list[bytes] = []

    def append(self, data) -> bool:
        self.parts.append(data if isinstance(data, bytes) else str(data).encode("utf-8", "surrogateescape"))
        return True

    write = append

    def build(self, filename: str) -> bool:
        self.fs.store_data(b"".join(self.parts), filename)
        self.parts = []
        return True


class cnn:  # noqa: N801
    _VERSION = "0.2"
    _NAME = "cnn"

    def __init__(self, connection_string: str | None = None, dbname: str = "tmp", auth_table=None):
        self.connection_string = connection_string
        self.dbname = dbname
        self.gridfs_dbname = dbname
        self.auth_table = auth_table
        self.db: Client | None = None
        self.pending_inserts: dict[str, list] = {}
        self.pending_callbacks: dict[str, list] = {}

    def connect(self) -> Client:
        if self.db is None:
            self.db = Client(split_endpoints(self.connection_string)[0])
        return self.db

    def gridfs(self) -> GridFS:
        eps = split_endpoints(self.connection_string)
        if len(eps) == 1:
            return GridFS(self.connect(), self.gridfs_dbname)
        if getattr(self, "_blob_clients", None) is None:
            self._blob_clients = [self.connect()] + [Client(e) for e in eps[1:]]
        return GridFS(self._blob_clients, self.gridfs_dbname)

    def grid_file_builder(self) -> GridFileBuilder:
        return GridFileBuilder(self.gridfs())

    def get_dbname(self) -> str:
        return self.dbname

    # -- error channel -------------------------------------------------------
    def insert_error(self, who: str, msg: str) -> None:
        self.connect().request("ERR_INSERT", self.dbname, who, msg)

    def get_errors(self) -> list[dict]:
        """Take (and remove) all pending error documents."""
        _, f = self.connect().request("ERR_TAKE", self.dbname)
        return [{"_id": i // 2, "worker": f[i].decode(), "msg": f[i + 1].decode("utf-8", "replace")}
                for i in range(0, len(f), 2)]

    def wait_change(self, since: int, timeout: float) -> int:
        """Block until the database has changed since mutation count ``since``
        (returned by an earlier call; -1 = return the current count now) or
        ``timeout`` seconds pass; returns the current mutation count."""
        _, f = self.connect().request("WAIT_CHANGE", self.dbname, since, max(0.0, timeout) * 1000.0)
        return int(f[0])

    def remove_errors(self, ids) -> None:
        # errors are removed atomically by get_errors (ERR_TAKE)
        return None

    # -- batched inserts -------------------------------------------------------
    def annotate_insert(self, ns: str, tbl: dict, callback: Callable | None = None) -> None:
        self.pending_inserts.setdefault(ns, []).append(tbl)
        cbs = self.pending_callbacks.setdefault(ns, [])
        if callback:
            cbs.append(callback)
        if len(self.pending_inserts[ns]) >= utils.MAX_PENDING_INSERTS:
            self._insert_batch(ns, self.pending_inserts[ns])
            for i, f in enumerate(self.pending_callbacks[ns]):
                f(self.pending_inserts[ns][i])
            self.pending_inserts[ns] = []
            self.pending_callbacks[ns] = []

    def flush_pending_inserts(self, max_pending: int = 0) -> None:
        for ns, tbl in list(self.pending_inserts.items()):
            if len(tbl) > max_pending:
                self._insert_batch(ns, tbl)
                for i, f in enumerate(self.pending_callbacks.get(ns, [])):
                    f(tbl[i])
        self.pending_inserts = {}
        self.pending_callbacks = {}

    def _insert_batch(self, ns: str, docs: list[dict]) -> None:
        """Insert documents in requests of up to 4096 jobs each (duplicates
        are skipped, as a unique index would reject them)."""
        c = self.connect()
        for a in range(0, len(docs), 4096):
            fields = []
            for d in docs[a:a + 4096]:
                fields += [d["_id"], json.dumps(d.get("value")), d.get("creation_time", utils.time())]
            c.request("JOB_INSERT", self.dbname, ns, *fields)

    # -- job collections (the <db>.map_jobs / <db>.red_jobs namespaces) -------
    def jobs(self, ns: str) -> "JobCollection":
        return JobCollection(self.connect(), self.dbname, ns)


def status_mask(*statuses: int) -> int:
    m = 0
    for s in statuses:
        m |= 1 << s
    return m


class JobCollection:
    def __init__(self, client: Client, dbname: str, ns: str):
        self.c, self.db, self.ns = client, dbname, ns

    def insert(self, job: dict) -> bool:
        st, _ = self.c.request("JOB_INSERT", self.db, self.ns, job["_id"], json.dumps(job["value"]),
                               job.get("creation_time", utils.time()))
        return st == 0

    def remove_status(self, *statuses: int) -> int:
        return int(self.c.request("JOB_REMOVE_STATUS", self.db, self.ns, status_mask(*statuses))[1][0])

    def fail_broken(self, max_reps: int) -> int:
        return int(self.c.request("JOB_FAIL_BROKEN", self.db, self.ns, max_reps)[1][0])

    def count(self, *statuses: int) -> int:
        return int(self.c.request("JOB_COUNT", self.db, self.ns, status_mask(*statuses))[1][0])

    def claim(self, worker: str, tmpname: str, t: float, statuses=(0, 2), only_ids=None,
              wait: float = 0.0) -> dict | None:
        """Claim one job atomically.  ``wait`` > 0 (seconds): a long poll —
        when nothing is claimable the coordinator holds the request until a
        job can be claimed, the task document changes, or ``wait`` expires."""
        ids = list(only_ids) if only_ids else []
        if only_ids is not None and not ids:
            return None
        if wait > 0:
            st, f = self.c.request("JOB_CLAIM_WAIT", self.db, wait * 1000.0, self.ns, worker, tmpname, t,
                                   status_mask(*statuses), *ids)
        else:
            st, f = self.c.request("JOB_CLAIM", self.db, self.ns, worker, tmpname, t, status_mask(*statuses), *ids)
        return decode_jobs(f)[0] if st == 0 else None

    def update(self, job_id: str, guard_tmpname: str = "", **fields) -> dict | None:
        args = []
        for k, v in fields.items():
            args += [k, v]
        st, f = self.c.request("JOB_UPDATE", self.db, self.ns, job_id, guard_tmpname, *args)
        return decode_jobs(f)[0] if st == 0 else None

    def get(self, job_id: str) -> dict | None:
        st, f = self.c.request("JOB_GET", self.db, self.ns, job_id)
        return decode_jobs(f)[0] if st == 0 else None

    def list(self) -> list[dict]:
        return decode_jobs(self.c.request("JOB_LIST", self.db, self.ns)[1])

    def drop(self) -> None:
        self.c.request("JOB_DROP", self.db, self.ns)

    def stats(self) -> dict:
        f = self.c.request("JOB_STATS", self.db, self.ns)[1]
        return {"sum_cpu_time": float(f[0]), "sum_real_time": float(f[1]), "real_time": float(f[2]),
                "counts": [int(x) for x in f[3:9]]}

    def expire(self, now: float, lease: float) -> int:
        return int(self.c.request("JOB_EXPIRE", self.db, self.ns, now, lease)[1][0])


def utest(connection_string=None) -> None:
    """cnn.lua:119-161: connection, blob store + builder, the error channel and
    batched inserts flushed at MAX_PENDING_INSERTS with per-document callbacks."""
    c = cnn(connection_string, "test")
    assert c.connect() is not None and c.get_dbname() == "test"
    g = c.gridfs()
    b = c.grid_file_builder()
    b.append(b"hello ")
    b.append(b"world")
    g.remove_file("cnn_utest")
    b.build("cnn_utest")
    assert g.get("cnn_utest") == b"hello world"
    g.remove_file("cnn_utest")
    assert g.get("cnn_utest") is None
    c.get_errors()
    c.insert_error("w1", "msg1")
    c.insert_error("w2", "msg2")
    errs = c.get_errors()
    assert [(e["worker"], e["msg"]) for e in errs] == [("w1", "msg1"), ("w2", "msg2")]
    assert c.get_errors() == []
    ns = "cnn_utest_jobs"
    c.jobs(ns).drop()
    seen = []
    old = utils.MAX_PENDING_INSERTS
    utils.MAX_PENDING_INSERTS = 50
    try:
        for i in range(120):
            c.annotate_insert(ns, utils.make_job(i, {"v": i}), lambda doc: seen.append(doc["_id"]))
        assert c.jobs(ns).count() == 100 and len(seen) == 100  # two automatic flushes
        c.flush_pending_inserts(0)
        assert c.jobs(ns).count() == 120 and len(seen) == 120
    finally:
        utils.MAX_PENDING_INSERTS = old
    c.jobs(ns).drop()
