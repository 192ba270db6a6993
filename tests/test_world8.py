"""World size 8 — the one-node target (8 x MI355X) — rehearsed with 8 gloo
ranks on CPU for every data plane: fold (word count), list (inverted index),
record (skewed TeraSort-style rows, range partitioner) and general (the
host combiner + reducefn, and typed folds), each with num_reducers in
{4, 10, 15}: fewer partitions than ranks (ranks that own no partition),
and counts not divisible by W.  Reference: reduce jobs exist only for the
partitions present (/root/reference/mapreduce/server.lua:279-326); partition p
is reduced by rank p % W here."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

W8 = 8
NREDS = (4, 10, 15)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _text():
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    return europarl_like(seed=21, lines=4000, words=60_000, vocab_size=4000, split_lines=250)


def _gather_pairs(eng, res) -> dict:
    from lua_mapreduce_1_amd.runtime import codec
    out = {}
    for _n, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            out[k] = list(v)
    return out


def _fold(R, device):
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    M = "lua_mapreduce_1_amd.models.wordcount"
    splits = _text()
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                    init_args={"nsplits": len(splits), "num_reducers": R}), device=device,
               split_store=SplitStore(splits, pin=False))
    res = eng.run()
    got = _gather_pairs(eng, res)
    naive: dict = {}
    for s in splits:
        for w in s.split():
            k = w.decode()
            naive[k] = naive.get(k, 0) + 1
    return res, lambda: got == {k: [v] for k, v in naive.items()}


def _list(R, device):
    import importlib
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    M = "lua_mapreduce_1_amd.examples.InvertedIndex"
    splits = _text()
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                    init_args={"nsplits": len(splits), "num_reducers": R}, table_capacity=1 << 14),
               device=device, split_store=SplitStore(splits, pin=False))
    res = eng.run()
    mod = importlib.import_module(M)
    return res, lambda: mod.RESULT == mod.naive_index(splits)


def _records(R, device):
    from lua_mapreduce_1_amd import spmd
    from test_records import check
    args = dict(rb=24, kb=3, skew=True, rows=24_000, blocks=W8 * 2, partitions=R)
    M = "rec_modules"
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, init_args=dict(args)), device=device)
    res = eng.run_iteration()
    parts = eng.gather_results(res)
    rows = np.concatenate([c["records"] for _n, c in parts]) if parts else None
    return res, lambda: rows is not None and check(rows, args)


def _generic(R, device):
    from test_generic_plane import close_lists, run_engine
    import comb_modules
    splits = _text()
    eng, res, got = run_engine("comb_modules", splits, device, {"mode": "host", "num_reducers": R})
    return res, lambda: close_lists(got, comb_modules.oracle(splits, "host"))


def _generic_cols(R, device):
    from test_generic_plane import close_lists, run_engine
    from lua_mapreduce_1_amd.utils.corpus import score_csv
    import importlib
    splits = score_csv(seed=5, lines=16_000, vocab_size=1200, split_lines=500)
    SS = "lua_mapreduce_1_amd.examples.ScoreStats"
    eng, res, got = run_engine(SS, splits, device, {"num_reducers": R})
    return res, lambda: close_lists(got, importlib.import_module(SS).naive(splits))


def _list_rounds(R, device):
    """The list plane with reduce rounds (reduce_cap_mb) after the shuffle."""
    import importlib
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    M = "lua_mapreduce_1_amd.examples.InvertedIndex"
    splits = _text()
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, reduce_cap_mb=0.01,
                    init_args={"nsplits": len(splits), "num_reducers": R}, table_capacity=1 << 14),
               device=device, split_store=SplitStore(splits, pin=False))
    res = eng.run()
    mod = importlib.import_module(M)
    return res, lambda: mod.RESULT == mod.naive_index(splits)


def _generic_rounds(R, device):
    from test_generic_plane import close_lists, run_engine
    import comb_modules
    splits = _text()
    eng, res, got = run_engine("comb_modules", splits, device, {"mode": "topk", "num_reducers": R},
                               reduce_cap_mb=0.01)
    return res, lambda: close_lists(got, comb_modules.oracle(splits, "topk"))


def _host(R, device):
    """The host plane (plain mapfn, no device_mapfn): the reference's tuple
    keys and values through the SPMD engine's host shuffle."""
    from lua_mapreduce_1_amd import spmd
    import host_modules as H
    M = "host_modules"
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, init_args={"num_reducers": R}),
               device=device)
    res = eng.run()
    return res, lambda: H.RESULT == H.naive(H._SPLITS)


def _value_rows(mod, splits, R, device):
    """Tuple values (PositionalIndex) / byte-string values (SourceIndex) on
    the general plane's value lists."""
    import importlib
    from test_generic_plane import run_engine
    eng, res, got = run_engine(mod, splits, device, {"num_reducers": R})
    exp = importlib.import_module(mod).naive(splits)
    if mod.endswith("PositionalIndex"):
        got = {k: [tuple(v) for v in vs] for k, vs in got.items()}
    return res, lambda: got == exp


def _positional(R, device):
    return _value_rows("lua_mapreduce_1_amd.examples.PositionalIndex", _text(), R, device)


def _sources(R, device):
    from lua_mapreduce_1_amd.examples import SourceIndex
    return _value_rows("lua_mapreduce_1_amd.examples.SourceIndex", SourceIndex.corpus(seed=4, lines=4000), R, device)


PLANES = {"host": _host, "positional": _positional, "sources": _sources, "fold": _fold, "list": _list, "records": _records, "generic": _generic, "generic_cols": _generic_cols,
          "list_rounds": _list_rounds, "generic_rounds": _generic_rounds}


def _rank(rank, world, port, q, plane):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_NUMA_BIND="0")
    torch.set_num_threads(1)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    _, _, device = D.init_from_env(backend="gloo", use_gpu=False)
    out = []
    for R in NREDS:
        res, ok = PLANES[plane](R, device)
        owned = sorted(int(p) for p in res.result_names)
        own_ok = all(p % world == rank for p in owned) and all(p < R for p in owned)
        allowned = D.gather_objects(owned, 0)
        if rank == 0:
            parts = sorted(p for o in allowned for p in o)
            out.append((R, bool(ok()), own_ok, parts == sorted(set(parts)), len(parts)))
        else:
            out.append((R, True, own_ok, True, 0))
    oks = D.gather_objects(all(o[2] for o in out), 0)
    if rank == 0:
        q.put((out, all(oks)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("plane", list(PLANES))
def test_world8_gloo(plane):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, W8, port, q, plane)) for r in range(W8)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    out, own = q.get(timeout=5)
    assert own, "a rank reduced a partition it does not own"
    for R, ok, _o, distinct, nparts in out:
        assert ok, (plane, R)
        assert distinct and 0 < nparts <= R, (plane, R, nparts)
