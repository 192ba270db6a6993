"""Host reducers recognised as device folds (parallel/recognize.py): the
reference's default contract (a per-key ``reducefn``, WordCount reducefn2 —
/root/reference/mapreduce/examples/WordCount/reducefn2.lua, test.sh:37-53)
run batched over every key's list instead of Python per key."""
import dataclasses
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lua_mapreduce_1_amd.parallel import recognize as RZ  # noqa: E402


def r_sum(key, values, emit):
    emit(sum(values))


def r_min(k, vs, emit):
    """docstring is fine"""
    emit(min(vs))


def r_max(k, vs, out):
    out(max(vs))


def r_loop(key, values, emit):
    acc = 0
    for v in values:
        acc += v
    emit(acc)


def r_loop2(key, values, emit):
    total = 0
    for x in values:
        total = x + total
    emit(total)


def n_mean(key, values, emit):
    emit(sum(values) / len(values))


def n_two(key, values, emit):
    emit(sum(values))
    emit(len(values))


def n_side(key, values, emit):
    print(key)
    emit(sum(values))


def n_start(key, values, emit):
    emit(sum(values, 10))


def n_other(key, values, emit):
    emit(sum(key))


def n_loop_mul(key, values, emit):
    acc = 0
    for v in values:
        acc *= v
    emit(acc)


def n_loop_init(key, values, emit):
    acc = 1
    for v in values:
        acc += v
    emit(acc)


def n_default(key, values, emit=print):
    emit(sum(values))


def _shadow_module():
    g = {"__builtins__": __builtins__, "sum": lambda xs: 42}
    exec("def f(key, values, emit):\n    emit(sum(values))\n", g)
    return g["f"]


@pytest.mark.parametrize("fn,want", [(r_sum, "sum"), (r_min, "min"), (r_max, "max"), (r_loop, "sum"),
                                     (r_loop2, "sum"), (n_mean, None), (n_two, None), (n_side, None),
                                     (n_start, None), (n_other, None), (n_loop_mul, None),
                                     (n_loop_init, None), (n_default, None), (len, None), (None, None)])
def test_recognize_patterns(fn, want):
    assert RZ.recognize(fn) == want


def test_recognize_shadowed_builtin():
    # exec'd source has no file: not recognised (no source), and a shadowed sum never is
    assert RZ.recognize(_shadow_module()) is None


def test_device_fold_exactness():
    off = torch.tensor([0, 2, 5])
    val = torch.tensor([3, 4, -1, 7, 2])
    assert RZ.device_fold("sum", "i64")(None, off, val).tolist() == [7, 8]
    assert RZ.device_fold("min", "i64")(None, off, val).tolist() == [3, -1]
    assert RZ.device_fold("max", "f64")(None, off, val.double()).tolist() == [4.0, 7.0]
    assert RZ.device_fold("sum", "f64") is None  # order-dependent rounding: stays on the host


def test_list_reducers_pick_recognised_folds(monkeypatch):
    import types
    from lua_mapreduce_1_amd.parallel import reducers as RD
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    mod = types.SimpleNamespace(reducefn=r_sum, combinerfn=r_sum)
    lr = RD.ListReducers(mod, "i64")
    assert lr.recognized == {"reducefn": "sum"} and lr.device_reduce and lr.device_combinerfn is lr.device_reducefn
    mod2 = types.SimpleNamespace(reducefn=n_mean, combinerfn=r_loop)
    lr2 = RD.ListReducers(mod2, "i64")
    assert lr2.recognized == {"combinerfn": "sum"} and not lr2.device_reduce
    assert RD.ListReducers(types.SimpleNamespace(reducefn=r_sum), "f64").recognized == {}
    assert RD.ListReducers(types.SimpleNamespace(reducefn=r_sum), ("i64", "i64")).recognized == {}
    monkeypatch.setattr(RD, "TUNABLES", dataclasses.replace(TUNABLES, recognize_reducers=False))
    assert RD.ListReducers(mod, "i64").recognized == {}


def test_reducefn2_wordcount_recognised_cpu(monkeypatch):
    """WordCount with reducefn2 (no hooks, no flags) on the general plane:
    the same counts with the fold recognised (no per-key host call) as with
    the host path."""
    import dataclasses as dc
    from lua_mapreduce_1_amd.parallel import reducers as RD
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    from test_generic_plane import make_data
    splits = make_data("text")[:3]
    W = "lua_mapreduce_1_amd.examples.WordCount"
    out = {}
    for recognize in (True, False):
        monkeypatch.setattr(RD, "TUNABLES", dc.replace(TUNABLES, recognize_reducers=recognize))
        eng = SPMDEngine(dict(taskfn=W, mapfn=W, partitionfn=W, reducefn=W + ".reducefn2", finalfn=None,
                              init_args={"nsplits": len(splits)}),
                         split_store=SplitStore(splits, pin=False), device=torch.device("cpu"))
        res = eng.run()
        assert eng.plane_kind == "generic"
        out[recognize] = {k: list(v) for _n, cols in eng.gather_results(res) for k, v in codec.iter_columnar(cols)}
        assert eng.plane.map.reducers.recognized == ({"reducefn": "sum"} if recognize else {})
    assert out[True] == out[False] and len(out[True]) > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("red", ["reducefn2", "reducefn3"])
def test_wordcount_general_reducers_gpu(red):
    """GPU: WordCount with reducefn2 (recognised sum: run-length postings
    combined from their counts) and reducefn3 (explicit device_reducefn over
    lists built from the counts) against the CPU host path, also through a
    forced one-rank shuffle (the receive table keeps plain postings)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from test_generic_plane import make_data
    splits = make_data("text")
    W = "lua_mapreduce_1_amd.examples.WordCount"
    out = {}
    for dev in ("cpu", "cuda"):
        eng = SPMDEngine(dict(taskfn=W, mapfn=W, partitionfn=W, reducefn=W + "." + red, finalfn=None,
                              init_args={"nsplits": len(splits)}),
                         split_store=SplitStore(splits, pin=dev == "cuda"), device=torch.device(dev))
        for _ in range(2):  # the second iteration reuses the map tables
            res = eng.run()
        out[dev] = {k: list(v) for _n, cols in eng.gather_results(res) for k, v in codec.iter_columnar(cols)}
        if dev == "cuda":
            mp = eng.plane.map
            assert mp.combines >= 1
            assert (mp.reducers.combiner_fold == "sum") == (red == "reducefn2")
    assert out["cpu"] == out["cuda"] and len(out["cpu"]) > 1000
