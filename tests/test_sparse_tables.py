"""Sparse map tables (parallel/spmd.py, MR_MAP_SPARSITY / MR_MAP_SPARSE_MIN_MB):
after a map of a large enough share, the engine sizes the next maps' tables
at `map_sparsity` slots per distinct key; the results stay those of the
first iteration (CPU engine; the GPU path is covered by
test_ops_gpu.py::test_spmd_prefetch_pipelined_iterations_match)."""
import dataclasses

import pytest

from lua_mapreduce_1_amd.parallel import spmd as S
from lua_mapreduce_1_amd.runtime import codec
from lua_mapreduce_1_amd.utils.corpus import europarl_like

M = "lua_mapreduce_1_amd.models.wordcount"


def _run(monkeypatch, min_mb):
    monkeypatch.setattr(S, "TUNABLES", dataclasses.replace(S.TUNABLES, map_sparse_min_mb=min_mb, map_sparsity=64))
    splits = europarl_like(seed=4, lines=4000, words=60_000, vocab_size=30_000, split_lines=500)
    eng = S.SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                            init_args={"nsplits": len(splits), "num_reducers": 4}),
                       split_store=S.SplitStore(splits, pin=False), device="cpu", table_capacity=1 << 12)
    out = []
    for _ in range(3):
        r = eng.run_iteration()
        out.append({k: v[0] for _n, cols in eng.gather_results(r) for k, v in codec.iter_columnar(cols)})
    return eng, out


def test_tables_grow_after_a_large_map_and_results_stay_exact(monkeypatch):
    eng, out = _run(monkeypatch, 0.0)
    assert sum(out[0].values()) == 60_000
    assert out[0] == out[1] == out[2]
    assert eng._table_capacity >= 64 * len(out[0])
    assert eng.table.cap == eng._table_capacity  # the table in use was replaced by a sparse one


def test_small_shares_keep_their_table(monkeypatch):
    eng, out = _run(monkeypatch, 1024.0)
    assert out[0] == out[2]
    assert eng._table_capacity < 64 * len(out[0])  # only the overflow regrowth, no sparsity


@pytest.mark.gpu
def test_overflowed_table_is_fitted_for_later_maps_gpu(gpu):
    """A first map that overflows its table (6 k keys, 4 k slots) re-runs in a
    table grown 16x; the later maps get one fitted to the key count
    (2 slots per key, power of two), and every iteration's counts are exact."""
    splits = europarl_like(seed=5, lines=8000, words=200_000, vocab_size=6_000, split_lines=1000)
    eng = S.SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                            init_args={"nsplits": len(splits), "num_reducers": 4}),
                       split_store=S.SplitStore(splits), device=gpu, table_capacity=1 << 12)
    want = {}
    for s in splits:
        for w in s.split():
            want[w.decode()] = want.get(w.decode(), 0) + 1
    caps = []
    for _ in range(3):
        r = eng.run_iteration()
        got = {k: v[0] for _n, cols in eng.gather_results(r) for k, v in codec.iter_columnar(cols)}
        assert got == want
        caps.append(eng.table.cap)
    if len(want) <= 1 << 12:
        pytest.skip("corpus too small to overflow")
    assert caps[0] == 16 << 12  # grown 16x after the overflow
    assert caps[2] == 1 << (2 * len(want) - 1).bit_length()  # fitted: next_pow2(2 n)


def test_big_tables_come_down_to_their_fit():
    """A map table of 2^24 slots or more comes down to next_pow2(2 n) from
    twice that (the reset and the compaction stream every slot); smaller ones
    keep the 4x hysteresis; a fitted big table stays put."""
    from types import SimpleNamespace

    from lua_mapreduce_1_amd.parallel import spmd as S

    def eng(cap, mapped_mb):
        return SimpleNamespace(table=SimpleNamespace(cap=cap), _table_capacity=cap, _initial_capacity=1 << 20,
                               _mapped_bytes=mapped_mb << 20)
    e = eng(1 << 27, 300)  # 23 M bigram keys after the 4x regrowth
    S.SPMDEngine._adapt_capacity(e, 23_000_000)
    assert e._table_capacity == 1 << 26
    e.table.cap = e._table_capacity
    S.SPMDEngine._adapt_capacity(e, 23_000_000)
    assert e._table_capacity == 1 << 26
    small = eng(1 << 22, 0)
    S.SPMDEngine._adapt_capacity(small, 600_000)
    assert small._table_capacity == 1 << 22
