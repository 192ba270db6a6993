"""Pluggable intermediate storage (reference: mapreduce/fs.lua).

``router(cnn, hostnames, storage, path)`` returns ``(fs, make_builder,
make_lines_iterator)`` exactly like fs.lua:185-208:

* ``gridfs`` — blobs in the coordinator (the GridFS replacement);
* ``shared`` — a directory on a shared file system; builders publish with
  tmpfile + atomic rename (fs.lua:80-115);
* ``sshfs``  — mappers write locally, reducers pull the partition's files from
  each mapper host with ``scp -CB`` (fs.lua:141-181); falls back to ``shared``
  when all mappers are local or no hostnames are given (fs.lua:200-201);
* ``hbm``    — new: node-local files that stay in device memory
  (runtime/hbm_store.py): the coordinator holds a descriptor per file, the
  bytes stay in the map worker's exported HBM arena and reducers pull them
  peer to peer; works across the worker processes of one node.

``make_lines_iterator(name)`` yields decoded ``(key, [values])`` records.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile
import threading

from .. import utils
from . import codec


def make_wildcard_from_mongo_match(match_tbl) -> str:
    """Regex of a mongo-style match -> shell wildcard (fs.lua:35-38)."""
    rx = match_tbl["filename"]["$regex"] if isinstance(match_tbl, dict) else match_tbl
    return rx.replace("\\.", ".").replace(".*", "*").replace("^", "").replace("$", "")


def _rx(match):
    if match is None:
        return None
    if isinstance(match, dict):
        match = match["filename"]["$regex"]
    return re.compile(match)


class FileBuilder:
    """tmpfile + atomic rename publisher (fs.lua:80-115)."""

    def __init__(self):
        self.parts: list[bytes] = []

    def append(self, data) -> bool:
        self.parts.append(data if isinstance(data, bytes) else str(data).encode("utf-8", "surrogateescape"))
        return True

    write = append

    def build(self, path: str) -> bool:
        d = os.path.dirname(path)
        if not d:
            raise ValueError(f"Given an incorrect path '{path}'")
        os.makedirs(d, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp_")
        with os.fdopen(fd, "wb") as f:
            for p in self.parts:
                f.write(p)
        os.replace(tmp, path)
        self.parts = []
        return True


class SharedFS:
    def __init__(self, path: str, hostnames=None):
        self.path = path
        os.makedirs(path, exist_ok=True)

    def list(self, match=None) -> list[dict]:
        rx = _rx(match) or re.compile("^" + re.escape(self.path) + "/.*")
        out = []
        for root, _dirs, files in os.walk(self.path):
            for fn in files:
                if fn.startswith(".tmp_"):
                    continue
                full = os.path.join(root, fn)
                if rx.search(full):
                    out.append({"filename": full})
        out.sort(key=lambda d: d["filename"])
        return out

    def remove_file(self, filename: str) -> bool:
        return utils.remove(filename)

    def read(self, filename: str) -> bytes:
        with open(filename, "rb") as f:
            return f.read()


class SSHFS(SharedFS):
    """Local writes, ``scp -CB`` pulls from remote mapper hosts."""

    def __init__(self, path: str, hostnames):
        self.path = path.rstrip("/")
        self.tmpname = tempfile.mkdtemp(prefix="lua_sshfs_")
        self.hostnames = list(hostnames or [])
        self.local = utils.get_hostname()

    def list(self, match=None) -> list[dict]:
        rx_src = match["filename"]["$regex"] if isinstance(match, dict) else (match or f"{self.path}/.*")
        wildcard = make_wildcard_from_mongo_match(rx_src)
        done = set()
        for h in self.hostnames:
            if h in done or h in (self.local, "localhost", "127.0.0.1", utils.DEFAULT_HOSTNAME):
                continue
            done.add(h)
            r = subprocess.run(["scp", "-CB", f"{h}:{wildcard}", self.tmpname + "/"], capture_output=True)
            if r.returncode != 0:
                raise RuntimeError(f"Impossible to SCP remote files from {h}:{wildcard}")
        rx = re.compile(rx_src)
        out = []
        # local files (mappers on this host) and pulled copies
        if os.path.isdir(self.path):
            out += [{"filename": os.path.join(self.path, f)} for f in os.listdir(self.path)
                    if rx.search(os.path.join(self.path, f))]
        rx_tmp = re.compile(rx_src.replace(self.path, self.tmpname))
        out += [{"filename": os.path.join(self.tmpname, f)} for f in os.listdir(self.tmpname)
                if rx_tmp.search(os.path.join(self.tmpname, f))]
        out.sort(key=lambda d: d["filename"])
        return out

    def __del__(self):
        shutil.rmtree(getattr(self, "tmpname", ""), ignore_errors=True)


class HBMFS:
    """``hbm`` storage: the coordinator's blob store holds a descriptor per
    file (runtime/hbm_store.py), the bytes stay in the writer's device arena.
    Listing and removal are the coordinator's; reads resolve the descriptor."""

    def __init__(self, cnn, gen=None):
        self.g = cnn.gridfs()
        self.gen = gen

    def list(self, match=None, prefix: str = "") -> list[dict]:
        return self.g.list(match, prefix=prefix)

    def remove_file(self, filename: str) -> bool:
        return self.g.remove_file(filename)

    def get(self, filename: str) -> bytes | None:
        from . import hbm_store
        d = self.g.get(filename)
        if d is None or not hbm_store.is_descriptor(d):
            return d
        return hbm_store.store().read_bytes(d)

    read = get


class HBMBuilder:
    def __init__(self, fs: HBMFS):
        self.fs = fs
        self.parts: list[bytes] = []

    def append(self, data) -> bool:
        self.parts.append(data if isinstance(data, bytes) else str(data).encode("utf-8", "surrogateescape"))
        return True

    write = append

    def build(self, filename: str) -> bool:
        from . import hbm_store
        (name, desc), = hbm_store.store().put_many([(filename, b"".join(self.parts))], self.fs.gen)
        self.fs.g.store_many([(name, desc)])
        self.parts = []
        return True


def router(cnn, hostnames, storage: str, path: str, gen=None):
    """``gen``: the task iteration a writer's files belong to (``hbm``: the
    arena of an earlier iteration is released when the next one writes)."""
    if storage == "gridfs":
        g = cnn.gridfs()
        return g, (lambda: cnn.grid_file_builder()), (lambda name: codec.decode_records(g.get(name) or b""))
    if storage == "hbm":
        m = HBMFS(cnn, gen)
        return m, (lambda: HBMBuilder(m)), (lambda name: codec.decode_records(m.get(name) or b""))
    if storage == "sshfs" and hostnames:
        s = SSHFS(path, hostnames)

        def lines(name):
            if not os.path.exists(name):
                name = name.replace(s.path, s.tmpname)
            return codec.decode_records(s.read(name))
        return s, FileBuilder, lines
    if storage in ("shared", "sshfs"):
        s = SharedFS(path)
        return s, FileBuilder, (lambda name: codec.decode_records(s.read(name)))
    raise ValueError(f"Given incorrect storage {storage}")


def read_blob(cnn, storage: str, path: str, name: str) -> bytes:
    """Raw bytes of a stored file (used for columnar device files)."""
    if storage == "gridfs":
        return cnn.gridfs().get(name) or b""
    if storage == "hbm":
        return HBMFS(cnn).get(name) or b""
    with open(name, "rb") as f:
        return f.read()


def utest(connection_string=None) -> None:
    """fs.lua:213-251: wildcard conversion; for every storage write two files,
    list them, read them back, remove them (sshfs through local paths)."""
    from .cnn import cnn as cnn_cls
    assert make_wildcard_from_mongo_match({"filename": {"$regex": "^/tmp/a\\.P1\\..*$"}}) == "/tmp/a.P1.*"
    c = cnn_cls(connection_string, "test")
    base = tempfile.mkdtemp(prefix="mr_fs_utest_")
    try:
        for storage in ("gridfs", "shared", "sshfs", "hbm"):
            path = os.path.join(base, storage)
            fs, make_builder, lines = router(c, [utils.get_hostname()], storage, path)
            names = [f"{path}/fs_utest.P0.M1", f"{path}/fs_utest.P0.M2"]
            for i, name in enumerate(names):
                fs.remove_file(name)
                bld = make_builder()
                bld.append(codec.encode_records([("k%d" % i, [i])]))
                bld.build(name)
            got = sorted(f["filename"] for f in fs.list({"filename": {"$regex": "^" + re.escape(path) +
                                                                      r"/fs_utest\.P0\..*"}}))
            assert got == names, (storage, got)
            for i, name in enumerate(names):
                assert list(lines(name)) == [("k%d" % i, [i])]
                fs.remove_file(name)
            assert not fs.list({"filename": {"$regex": "^" + re.escape(path) + r"/fs_utest.*"}})
    finally:
        shutil.rmtree(base, ignore_errors=True)
