"""The general device plane in the reference's deployment shape (server +
workers over the coordinator): typed folds written as MRC2 partition files
and merged by the device reduce, value lists written as records for the
host reducefn, and the host plane of the same modules — all diffed against
the modules' oracles (CPU tensors here; GPU variants in test_generic_gpu.py)."""
import importlib
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lua_mapreduce_1_amd.runtime import coordinator  # noqa: E402
from test_e2e_wordcount import run_job  # noqa: E402
from test_generic_plane import close_lists, make_data, oracle  # noqa: E402

SS = "lua_mapreduce_1_amd.examples.ScoreStats"
BG = "lua_mapreduce_1_amd.examples.Bigram"
GM = "gen_modules"


@pytest.fixture(scope="module")
def cs():
    return coordinator.start_local()


def write(tmp_path, splits):
    paths = []
    for i, s in enumerate(splits):
        p = tmp_path / f"split{i:03d}.txt"
        p.write_bytes(s)
        paths.append(str(p))
    return paths


def job(cs, tmp_path, which, mod, args, plane, storage="gridfs", nworkers=2, db=""):
    splits = make_data(which)[:4]
    files = write(tmp_path, splits)
    p = dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod, finalfn=mod if mod != GM else GM,
             init_args=dict(args, files=files), storage=storage, device="auto" if plane == "device" else "host")
    _, s = run_job(cs, f"gen_{db}_{which}_{args.get('mode', '')}_{plane}_{storage}", p, nworkers=nworkers)
    got = importlib.import_module(mod).RESULT
    return got, oracle(which, args.get("mode"), splits), s


@pytest.mark.parametrize("plane", ["host", "device"])
@pytest.mark.parametrize("which,mod,args", [("scores", SS, {}), ("text", BG, {"mode": "bigram"}),
                                            ("text", GM, {"mode": "max_host"}), ("text", GM, {"mode": "docs"}),
                                            ("text", GM, {"mode": "mixed"})],
                         ids=["scores", "bigram", "max_host", "docs", "mixed"])
def test_generic_server_worker(cs, tmp_path, which, mod, args, plane):
    got, exp, s = job(cs, tmp_path, which, mod, args, plane)
    if mod == BG:
        got = {k: (v if isinstance(v, list) else [v]) for k, v in got.items()}
    assert close_lists(got, exp)
    assert s.last_stats["failed_map_jobs"] == 0 and s.last_stats["failed_red_jobs"] == 0


@pytest.mark.parametrize("storage", ["shared", "hbm"])
def test_generic_server_worker_storages(cs, tmp_path, storage):
    got, exp, _ = job(cs, tmp_path, "scores", SS, {}, "device", storage=storage, db=storage)
    assert close_lists(got, exp)
