"""sshfs storage pulling mapper output from other hosts with ``scp -CB``
(reference: /root/reference/mapreduce/fs.lua:142-175, the sshfs router branch at
fs.lua:191-199).  The container has no sshd, so ``scp`` is a stub on PATH
that serves ``host:/abs/pattern`` from a per-host directory tree and logs
its arguments: the test covers the command line, the wildcard, the pulled
copies' listing and reading through the router, de-duplicated hosts, local
hosts read in place, and a failing transfer."""
import os
import sys

import pytest

from lua_mapreduce_1_amd.runtime import codec
from lua_mapreduce_1_amd.runtime import fs as F
from lua_mapreduce_1_amd import utils

STUB = """#!{py}
import glob, os, shutil, sys
with open({log!r}, "a") as f:
    f.write(" ".join(sys.argv[1:]) + "\\n")
src, dst = sys.argv[-2], sys.argv[-1]
host, pat = src.split(":", 1)
if host == "deadhost":
    sys.exit(1)
for p in glob.glob(os.path.join({hosts!r}, host) + pat):
    shutil.copy(p, dst)
"""


@pytest.fixture
def scp_stub(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "scp.log"
    hosts = tmp_path / "hosts"
    stub = bindir / "scp"
    stub.write_text(STUB.format(py=sys.executable, log=str(log), hosts=str(hosts)))
    stub.chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ['PATH']}")
    return log, hosts


def _write(path: str, records) -> None:
    b = F.FileBuilder()
    b.append(codec.encode_records(records))
    b.build(path)


def test_sshfs_pulls_remote_mapper_files(tmp_path, scp_stub):
    log, hosts = scp_stub
    path = str(tmp_path / "job" / "results")
    # a mapper on nodeB wrote its partition files under the same path on its own disk
    remote_dir = str(hosts / "nodeB") + path
    _write(os.path.join(remote_dir, "map.P0.M1"), [("b", [2])])
    _write(os.path.join(remote_dir, "map.P0.M2"), [("c", [3])])
    _write(os.path.join(remote_dir, "map.P1.M1"), [("z", [9])])  # another partition: not pulled below
    # a mapper on this host wrote one locally
    _write(os.path.join(path, "map.P0.M0"), [("a", [1])])

    fsys, make_builder, lines = F.router(None, ["nodeB", "nodeB", utils.get_hostname()], "sshfs", path)
    assert isinstance(fsys, F.SSHFS)
    listed = fsys.list({"filename": {"$regex": "^" + path + "/map\\.P0\\..*$"}})
    names = [os.path.basename(d["filename"]) for d in listed]
    assert sorted(names) == ["map.P0.M0", "map.P0.M1", "map.P0.M2"]
    # one transfer for the de-duplicated remote host, none for the local one
    calls = log.read_text().splitlines()
    assert calls == [f"-CB nodeB:{path}/map.P0.* {fsys.tmpname}/"]
    got = {}
    for d in listed:
        for k, v in lines(d["filename"]):
            got[k] = v
    assert got == {"a": [1], "b": [2], "c": [3]}
    # remove_file deletes the pulled copies too
    for d in listed:
        assert fsys.remove_file(d["filename"])
    assert fsys.list({"filename": {"$regex": "^" + path + "/map\\.P0\\..*$"}}) == [
        {"filename": os.path.join(fsys.tmpname, "map.P0.M1")},
        {"filename": os.path.join(fsys.tmpname, "map.P0.M2")},
    ]  # listing pulls nodeB's files again (its disk still holds them), as the reference does


def test_sshfs_failed_transfer_raises(tmp_path, scp_stub):
    path = str(tmp_path / "job2")
    fsys, _b, _l = F.router(None, ["deadhost"], "sshfs", path)
    with pytest.raises(RuntimeError, match="Impossible to SCP remote files from deadhost"):
        fsys.list()
