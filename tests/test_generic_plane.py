"""The general device plane (parallel/generic.py): keys picked by user device
code (byte spans), typed / multi-column folds, int64 value lists, and the
module's own reducefn when it declares no device_reduce — on CPU tensors at
world size 1, forced shuffle, and gloo W = 3, against host oracles.  The GPU
variants are in test_generic_gpu.py."""
import math
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

SS = "lua_mapreduce_1_amd.examples.ScoreStats"
BG = "lua_mapreduce_1_amd.examples.Bigram"
GM = "gen_modules"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def close_lists(got: dict, exp: dict, rel: float = 1e-9) -> bool:
    if set(got) != set(exp):
        return False
    for k, e in exp.items():
        g = got[k]
        if len(g) != len(e):
            return False
        for a, b in zip(g, e):
            if isinstance(b, float) or isinstance(a, float):
                if not math.isclose(a, b, rel_tol=rel, abs_tol=1e-9):
                    return False
            elif a != b:
                return False
    return True


def make_data(which: str):
    from lua_mapreduce_1_amd.utils.corpus import europarl_like, score_csv
    if which == "scores":
        return score_csv(seed=3, lines=12_000, vocab_size=1500, split_lines=2000)
    return europarl_like(seed=5, lines=3000, words=30000, vocab_size=2500, split_lines=500)


def oracle(which: str, mode: str, splits):
    import importlib
    if which == "scores":
        return importlib.import_module(SS).naive(splits)
    if mode == "bigram":
        return {k: [v] for k, v in importlib.import_module(BG).naive(splits).items()}
    return importlib.import_module(GM).oracle(splits, mode)


def run_engine(mod, splits, device, args=None, **params):
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    init = dict(args or {}, nsplits=len(splits))
    eng = SPMDEngine(dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod, finalfn=None, init_args=init,
                          **params), split_store=SplitStore(splits, pin=device.type == "cuda"), device=device)
    res = eng.run()
    got = {}
    for _n, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            got[k] = list(v)
    return eng, res, got


CASES = [("scores", SS, {}), ("text", BG, {"mode": "bigram"}), ("text", GM, {"mode": "max_host"}),
         ("text", GM, {"mode": "docs"}), ("text", GM, {"mode": "docs_concat"}), ("text", GM, {"mode": "mixed"})]


@pytest.mark.parametrize("which,mod,args", CASES, ids=["scores", "bigram", "max_host", "docs", "docs_concat",
                                                       "mixed"])
def test_generic_cpu_w1(which, mod, args):
    splits = make_data(which)
    eng, res, got = run_engine(mod, splits, torch.device("cpu"), args)
    exp = oracle(which, args.get("mode"), splits)
    assert close_lists(got, exp)
    assert res.failed_maps == 0 and res.distinct_keys == len(exp)
    if mod == BG:
        assert eng.plane_kind == "fold"  # spans on the int64 fold plane
    else:
        assert eng.plane_kind == "generic"


def test_max_reducer_without_device_reduce_is_not_summed():
    """The silent-'sum' trap: a device map paired with a max reducefn and no
    device_reduce must return maxima (the reducefn runs per key)."""
    splits = make_data("text")
    _, _, got = run_engine(GM, splits, torch.device("cpu"), {"mode": "max_host"})
    exp = oracle("text", "max_host", splits)
    assert got == exp
    # the same data summed differs for repeated words: the test can tell
    acc = {}
    for k, v in __import__(GM).host_values(b"".join(s if s.endswith(b"\n") else s + b"\n" for s in splits)):
        acc[k] = acc.get(k, 0) + v
    assert any(acc[k] != exp[k][0] for k in exp)


def test_inverted_index_on_the_general_plane():
    """emit.word_lines through the general plane (plane='generic') equals the
    fused list plane's oracle."""
    from lua_mapreduce_1_amd.examples import InvertedIndex as II
    splits = make_data("text")
    eng, _, got = run_engine("lua_mapreduce_1_amd.examples.InvertedIndex", splits, torch.device("cpu"),
                             {"num_reducers": 4}, plane="generic")
    assert eng.plane_kind == "generic"
    assert got == II.naive_index(splits)


def test_word_lines_chunks_inside_splits():
    """emit.word_lines on the general plane with chunks that start inside a
    split: the chunk's line base (split base + the split's newlines before it)
    is formed on the device."""
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.examples import InvertedIndex as II
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    splits = make_data("text")
    M = "lua_mapreduce_1_amd.examples.InvertedIndex"
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, plane="generic",
                    init_args={"nsplits": len(splits), "num_reducers": 4}), device="cpu",
               split_store=SplitStore(splits, pin=False))
    eng.chunk_bytes = [5000]
    eng.tail_bytes = [5000]
    eng.run()
    assert eng.plane_kind == "generic"
    assert II.RESULT == II.naive_index(splits)


def test_list_plane_switches_to_generic_on_spans():
    """A concat_unique module whose map emits spans runs on the general plane
    (the list plane's fused emitter only knows word_lines)."""
    splits = make_data("text")
    eng, _, got = run_engine(GM, splits, torch.device("cpu"), {"mode": "docs"})
    assert eng.plane_kind == "generic"
    assert got == oracle("text", "docs", splits)


def test_pairs_rep_after_host_keys_many_chunks():
    """emit(host key) then emit.pairs(rep=...) in every one of many staged
    chunks: long keys of later chunks still point at their own bytes."""
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    splits = europarl_like(seed=13, lines=2000, words=20000, vocab_size=900, split_lines=100)
    splits = [s.replace(b" of ", b" extraordinarily_long_word_of_many_bytes ") for s in splits]
    eng = SPMDEngine(dict(taskfn=GM, mapfn=GM, partitionfn=GM, reducefn=GM, finalfn=None,
                          init_args={"mode": "pairs_host", "nsplits": len(splits)}),
                     split_store=SplitStore(splits, pin=False), device=torch.device("cpu"))
    eng.chunk_bytes = [8 << 10]
    eng.tail_bytes = [8 << 10]
    res = eng.run()
    got = {}
    for _n, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            got[k] = v[0]
    exp = {}
    for s in splits:
        for w in s.split():
            exp[w.decode()] = exp.get(w.decode(), 0) + 1
    nchunks = len(eng._chunks[0]) if eng._chunks[0] else None
    exp["__host_key__"] = got.get("__host_key__")
    assert got == exp
    assert got["__host_key__"] > 1, nchunks  # several chunks were mapped


def test_column_spec_parsing():
    from lua_mapreduce_1_amd.ops import agg as A
    assert [repr(c) for c in A.parse_spec(("f64:mean", "max", "count", "sum:f32"))] == [
        "f64:mean", "i64:max", "i64:count", "f32:sum"]
    assert A.is_column_spec("f64:sum") and A.is_column_spec(("sum", "max"))
    assert not A.is_column_spec("sum") and not A.is_column_spec("concat") and not A.is_column_spec(None)
    ph = A.Physical(A.parse_spec(("f64:mean", "count")))
    assert ph.cols == [("f64", "sum", 0), ("i64", "sum", None)]  # the mean and the count share the count
    assert ph.out == [("mean", 0, 1), ("col", 1)]
    with pytest.raises(ValueError):
        A.parse_spec("f64:median")


def test_unknown_device_reduce_raises():
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine
    mod = {"taskfn": lambda emit: None, "device_mapfn": lambda k, v, e: None, "device_reduce": "median",
           "partitionfn": lambda k: 0, "reducefn": lambda k, v, e: None}
    with pytest.raises(ValueError, match="unknown device_reduce"):
        SPMDEngine(dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod), device=torch.device("cpu"))


def test_text_ops_cpu():
    from lua_mapreduce_1_amd.ops import text as TX
    t = torch.frombuffer(bytearray(b"ab,1.5\n\ncd,-2e3\r\nxy\n  z , 7 \n"), dtype=torch.uint8)
    ls, ll = TX.lines(t)
    assert ls.tolist() == [0, 7, 8, 17, 20] and ll.tolist() == [6, 0, 8, 2, 8]
    ks, kl = TX.field(t, ls, ll, ",", 0)
    vs, vl = TX.field(t, ls, ll, ",", 1)
    assert kl.tolist() == [2, 0, 2, 2, 4] and vs.tolist()[3] == -1
    v = TX.parse_f64(t, vs, vl)
    assert v[0].item() == 1.5 and v[2].item() == -2000.0 and math.isnan(v[3].item()) and v[4].item() == 7.0
    st, ln = TX.tokens(t)
    assert [bytes(t[s:s + n].tolist()) for s, n in zip(st.tolist(), ln.tolist())] == [
        b"ab,1.5", b"cd,-2e3", b"xy", b"z", b",", b"7"]


# -- multi-rank (gloo) ---------------------------------------------------------
def _rank(rank, world, port, q, which, mod, args, force_shuffle):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import datetime
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    if force_shuffle:
        dist.init_process_group("gloo", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120))
    else:
        D.init_from_env(backend="gloo", use_gpu=False)
    splits = make_data(which)
    eng, res, got = run_engine(mod, splits, torch.device("cpu"), args, force_shuffle=force_shuffle)
    owned = sorted(res.partitions)
    ok_owned = all(p % world == rank for p in owned)
    stats = eng.stats_block(res)
    if rank == 0:
        exp = oracle(which, args.get("mode"), splits)
        q.put((close_lists(got, exp), ok_owned, len(got), stats))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, which, mod, args, force_shuffle=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, which, mod, args, force_shuffle))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return q.get(timeout=5)


@pytest.mark.parametrize("which,mod,args", CASES, ids=["scores", "bigram", "max_host", "docs", "docs_concat",
                                                       "mixed"])
def test_generic_gloo_w3(which, mod, args):
    ok, owned, n, _ = _spawn(3, which, mod, args)
    assert ok and owned and n > 100


@pytest.mark.parametrize("which,mod,args", [CASES[0], CASES[4]], ids=["scores", "docs_concat"])
def test_generic_forced_shuffle_w1(which, mod, args):
    ok, owned, n, _ = _spawn(1, which, mod, args, force_shuffle=True)
    assert ok and n > 100


def _long_text():
    from test_exactness import colliding_text
    return [colliding_text(11 + i, ntok=2000, nlong=150) for i in range(2)]


STREAM_CASES = [("scores", SS, {}), ("text", GM, {"mode": "max_host"}), ("text", GM, {"mode": "docs"}),
                ("text", GM, {"mode": "docs_concat"})]


@pytest.mark.parametrize("which,mod,args", STREAM_CASES, ids=["scores", "max_host", "docs", "docs_concat"])
def test_generic_streams_rounds_cpu(which, mod, args):
    """arena_cap_mb on the general plane: the rank's splits are mapped in
    rounds through the two capped ring slots, long keys moving to the key heap
    after each round; results equal the whole-input oracle."""
    splits = make_data(which) + (_long_text() if which == "text" else [])
    eng, res, got = run_engine(mod, splits, torch.device("cpu"), args, arena_cap_mb=0.06)
    assert eng.plane_kind == "generic"
    assert eng._streaming(eng._split_ids(eng._jobs(), 0, len(splits)))
    assert close_lists(got, oracle(which, args.get("mode"), splits))
    assert res.failed_maps == 0


def test_generic_streamed_host_keys_raise_cpu():
    with pytest.raises(ValueError, match="streamed general-plane map"):
        run_engine(GM, make_data("text"), torch.device("cpu"), {"mode": "mixed"}, arena_cap_mb=0.06)


@pytest.mark.parametrize("on_gpu", [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_generic_stream_heap_grows(request, monkeypatch, on_gpu):
    """A long-key heap too small for the rounds' long keys doubles and the
    general map re-runs; the value lists stay exact."""
    import dataclasses
    from test_exactness import colliding_text
    from lua_mapreduce_1_amd.parallel import generic as G
    from lua_mapreduce_1_amd.parallel import spmd as S
    from lua_mapreduce_1_amd.parallel import staging as ST
    dev = request.getfixturevalue("gpu") if on_gpu else torch.device("cpu")
    monkeypatch.setattr(S, "TUNABLES", dataclasses.replace(S.TUNABLES, stream_heap_mb=0.07))
    monkeypatch.setattr(ST, "TUNABLES", dataclasses.replace(ST.TUNABLES, stream_heap_mb=0.07))
    monkeypatch.setattr(G, "TUNABLES", dataclasses.replace(G.TUNABLES, stream_heap_mb=0.07))
    splits = [colliding_text(90 + i, ntok=20000, nlong=3000) for i in range(4)]
    cap = max(len(s) for s in splits) + 1
    eng, res, got = run_engine(GM, splits, dev, {"mode": "docs"}, arena_cap_mb=cap / (1 << 20))
    assert close_lists(got, oracle("text", "docs", splits))
    assert eng._stream_heap_mb > 0.07


@pytest.mark.gpu
@pytest.mark.parametrize("which,mod,args", STREAM_CASES, ids=["scores", "max_host", "docs", "docs_concat"])
def test_generic_streams_rounds_gpu(gpu, which, mod, args):
    splits = make_data(which) + (_long_text() if which == "text" else [])
    eng, res, got = run_engine(mod, splits, gpu, args, arena_cap_mb=0.06)
    assert eng._streaming(eng._split_ids(eng._jobs(), 0, len(splits)))
    assert close_lists(got, oracle(which, args.get("mode"), splits))
    assert res.failed_maps == 0


# -- split-level restart on the general plane ------------------
def _restart_rank(rank, world, port, q, which, mod, args, ckpt, fault):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_SPMD_FAULT=fault)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    D.init_from_env(backend="gloo", use_gpu=False, timeout_s=30)
    splits = make_data(which)
    eng, res, got = run_engine(mod, splits, torch.device("cpu"), args, checkpoint_dir=ckpt)
    if rank == 0:
        q.put((eng.maps_restored, close_lists(got, oracle(which, args.get("mode"), splits))))
    else:
        q.put((eng.maps_restored, None))
    dist.barrier()
    dist.destroy_process_group()


def _restart_launch(world, which, mod, args, ckpt, fault, expect_fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_restart_rank, args=(r, world, port, q, which, mod, args, ckpt, fault))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240 if not expect_fail else 120)
        if p.is_alive():
            p.terminate()
            p.join(10)
    if expect_fail:
        return [p.exitcode for p in procs], None
    return [p.exitcode for p in procs], [q.get(timeout=5) for _ in range(world)]


@pytest.mark.parametrize("which,mod,args", [CASES[0], CASES[3]], ids=["scores", "docs"])
def test_generic_restart_restores_map_outputs(tmp_path, which, mod, args):
    """Rank 1 dies after the map phase of iteration 1 (``1:1:exit::shuffle``):
    both ranks had checkpointed their map outputs (typed fold columns / value
    lists); the relaunch restores them instead of re-mapping, and the results
    equal the oracle."""
    ckpt = str(tmp_path / "ckpt")
    codes, _ = _restart_launch(2, which, mod, args, ckpt, "1:1:exit::shuffle", expect_fail=True)
    assert codes[1] == 17 and codes[0] != 0, codes
    assert len([f for f in os.listdir(ckpt) if ".map.it1." in f]) == 2
    codes, out = _restart_launch(2, which, mod, args, ckpt, "", expect_fail=False)
    assert codes == [0, 0], codes
    assert sorted(o[0] for o in out) == [1, 1]
    assert [o[1] for o in out if o[1] is not None] == [True]
    assert not [f for f in os.listdir(ckpt) if ".map." in f]  # consumed checkpoints are removed


def _restart_gpu_proc(q, which, mod, args, ckpt, fault):
    os.environ["MR_SPMD_FAULT"] = fault
    splits = make_data(which)
    eng, res, got = run_engine(mod, splits, torch.device("cuda", 0), args, checkpoint_dir=ckpt)
    q.put((eng.maps_restored, close_lists(got, oracle(which, args.get("mode"), splits))))


@pytest.mark.gpu
@pytest.mark.parametrize("which,mod,args", [CASES[0], CASES[3]], ids=["scores", "docs"])
def test_generic_restart_restores_map_outputs_gpu(gpu, tmp_path, which, mod, args):
    """One rank on the GPU exits after its map phase; the relaunch restores
    the saved map output into a fresh device table and the results are exact."""
    ckpt = str(tmp_path / "ckpt")
    ctx = mp.get_context("spawn")
    for fault, want_code in (("1:0:exit::shuffle", 17), ("", 0)):
        q = ctx.Queue()
        p = ctx.Process(target=_restart_gpu_proc, args=(q, which, mod, args, ckpt, fault))
        p.start()
        p.join(180)
        assert p.exitcode == want_code, p.exitcode
    restored, ok = q.get(timeout=5)
    assert restored == 1 and ok
