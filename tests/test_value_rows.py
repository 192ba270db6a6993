"""Tuple and byte-string values on the general device plane's value lists
(parallel/values.py): a positional inverted index with
(line, position) tuple values and a word -> distinct sources index with
byte-string values, against host oracles — CPU tensors at W = 1, forced
shuffle, gloo W = 3, plus the batched and host reducer hooks over such
values.  GPU variants: test_value_rows_gpu.py.  Reference: every emitted
value is a ``tuple(value)`` (/root/reference/mapreduce/job.lua:83-97),
serialised with its strings (utils.lua:100-120)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_generic_plane import _free_port, run_engine  # noqa: E402

PI = "lua_mapreduce_1_amd.examples.PositionalIndex"
SI = "lua_mapreduce_1_amd.examples.SourceIndex"


def pi_data():
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    return europarl_like(seed=7, lines=2400, words=24000, vocab_size=2000, split_lines=300)


def si_data():
    from lua_mapreduce_1_amd.examples import SourceIndex
    return SourceIndex.corpus(seed=3, lines=3000, split_lines=400)


def _pi_got(got):
    return {k: [tuple(v) for v in vs] for k, vs in got.items()}


def test_value_spec_and_host_bits():
    from lua_mapreduce_1_amd.parallel import values as VL
    sp = VL.ValueSpec(("i64", "f64", "bytes"))
    assert sp.width == 3 and sp.bytes_cols == [2] and not sp.scalar and sp.dtype == "tuple"
    assert VL.ValueSpec("i64").scalar and VL.ValueSpec("bytes").has_bytes
    with pytest.raises(ValueError):
        VL.ValueSpec("str")
    store = bytearray()

    def add(b):
        o = len(store)
        store.extend(b)
        return o
    bits = VL.host_bits([(1, 2.5, "ab"), (3, -1.0, "")], sp, add, "t")
    off = [0, 2, 2]
    import numpy as np
    vals = VL.host_columns(bits, sp, {2: (np.array(off), np.frombuffer(bytes(store), np.uint8))})
    assert vals == [(1, 2.5, "ab"), (3, -1.0, "")]
    with pytest.raises(TypeError):
        VL.host_bits([(1, 2.5)], sp, add, "t")


def test_positional_index_cpu():
    import importlib
    splits = pi_data()
    eng, res, got = run_engine(PI, splits, torch.device("cpu"), {"num_reducers": 7})
    assert eng.plane_kind in ("generic", "list")
    assert _pi_got(got) == importlib.import_module(PI).naive(splits)


def test_source_index_cpu():
    import importlib
    splits = si_data()
    eng, res, got = run_engine(SI, splits, torch.device("cpu"), {"num_reducers": 5})
    assert got == importlib.import_module(SI).naive(splits)


def _rank(rank, world, port, q, mod, which, args, params):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_NUMA_BIND="0")
    import importlib
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    D.init_from_env(backend="gloo", use_gpu=False)
    splits = pi_data() if which == "pi" else si_data()
    eng, res, got = run_engine(mod, splits, torch.device("cpu"), args, **params)
    exp = importlib.import_module(mod).naive(splits)
    if rank == 0:
        q.put((_pi_got(got) if which == "pi" else got) == exp)
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, mod, which, args, params=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, mod, which, args, params or {})) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return q.get(timeout=5)


@pytest.mark.parametrize("which", ["pi", "si"])
def test_value_rows_gloo_w3(which):
    mod = PI if which == "pi" else SI
    assert _spawn(3, mod, which, {"num_reducers": 7})


# -- hooks over tuple / byte values -------------------------------------------------
def test_host_reducefn_over_byte_values_cpu(monkeypatch):
    """No device_reduce: the module's reducefn runs per key over str values
    (and its combiner map-side over them)."""
    import importlib
    m = importlib.import_module(SI)
    monkeypatch.setattr(m, "device_reduce", None)
    calls = {"n": 0}

    def reducefn(key, values, emit):
        calls["n"] += 1
        assert all(isinstance(v, str) for v in values)
        for v in sorted(set(values), key=lambda x: x.encode("utf-8", "surrogateescape")):
            emit(v)
    monkeypatch.setattr(m, "reducefn", reducefn)
    monkeypatch.setattr(m, "combinerfn", reducefn)
    splits = si_data()
    eng, res, got = run_engine(SI, splits, torch.device("cpu"), {"num_reducers": 5})
    assert got == m.naive(splits) and calls["n"] > 0


def test_device_reducefn_over_tuples_cpu(monkeypatch):
    """device_reducefn receives the (line, position) rows as [n, 2] and
    returns per key (number of postings, first line)."""
    import importlib
    from lua_mapreduce_1_amd.ops import segments as S
    m = importlib.import_module(PI)
    monkeypatch.setattr(m, "device_reduce", None)
    monkeypatch.setattr(m, "combinerfn", None)
    seen = {}

    def device_reducefn(keys, off, val):
        seen["shape"] = tuple(val.shape)
        return S.count(off), S.min(off, val[:, 0].contiguous(), empty=0)
    monkeypatch.setattr(m, "device_reducefn", device_reducefn, raising=False)
    splits = pi_data()
    eng, res, got = run_engine(PI, splits, torch.device("cpu"), {"num_reducers": 7})
    exp = m.naive(splits)
    # the postings of a word, without a combiner: every (line, position) once
    assert {k: v for k, v in got.items()} == {k: [len(v), v[0][0]] for k, v in exp.items()}
    assert seen["shape"][1] == 2


def test_device_reducefn_over_bytes_cpu(monkeypatch):
    """device_reducefn receives ByteValues (CSR of the value bytes) and
    returns the number of distinct-length sources per key."""
    import importlib
    from lua_mapreduce_1_amd.parallel.values import ByteValues
    m = importlib.import_module(SI)
    monkeypatch.setattr(m, "device_reduce", None)
    monkeypatch.setattr(m, "combinerfn", None)

    def device_reducefn(keys, off, val):
        assert isinstance(val, ByteValues)
        lens = val.off[1:] - val.off[:-1]
        out = []
        o = off.tolist()
        for i in range(len(o) - 1):
            out.append(int(lens[o[i]:o[i + 1]].sum()))
        return torch.tensor(out, dtype=torch.int64)
    monkeypatch.setattr(m, "device_reducefn", device_reducefn, raising=False)
    splits = si_data()
    eng, res, got = run_engine(SI, splits, torch.device("cpu"), {"num_reducers": 5})
    occ: dict = {}
    for s in splits:
        for text in s.split(b"\n"):
            name, tab, rest = text.partition(b"\t")
            if not tab:
                name, rest = b"", name
            for w in rest.split():
                k = w.decode()
                occ[k] = occ.get(k, 0) + len(name)
    assert got == {k: [v] for k, v in occ.items()}


# -- the reference's deployment shape (server + workers over the coordinator) ---------
@pytest.mark.parametrize("plane", ["host", "device"])
@pytest.mark.parametrize("which", ["pi", "si"])
def test_value_rows_server_worker(tmp_path, which, plane):
    """Both examples through server/worker: the host plane (MRK1 records of
    tuples / strings) and the device map (value rows written as records for
    the reduce jobs), diffed against the oracles."""
    import importlib
    from lua_mapreduce_1_amd.runtime import coordinator
    from test_e2e_wordcount import run_job
    mod = PI if which == "pi" else SI
    splits = (pi_data() if which == "pi" else si_data())[:4]
    files = []
    for i, s in enumerate(splits):
        p = tmp_path / f"split{i}.txt"
        p.write_bytes(s)
        files.append(str(p))
    cs = coordinator.start_local()
    params = dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod, finalfn=mod,
                  init_args={"files": files, "num_reducers": 5}, storage="gridfs",
                  device="auto" if plane == "device" else "host")
    _, s = run_job(cs, f"vr_{which}_{plane}", params, nworkers=2)
    m = importlib.import_module(mod)
    got = _pi_got(m.RESULT) if which == "pi" else m.RESULT
    assert got == m.naive(splits)
    assert s.last_stats["failed_map_jobs"] == 0 and s.last_stats["failed_red_jobs"] == 0
