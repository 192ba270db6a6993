"""The per-module unit tests run through the aggregator (reference:
mapreduce/test.lua, which test.sh runs first)."""
from lua_mapreduce_1_amd import test as agg


def test_module_utests():
    agg.run()


def test_tuple_interning_is_weak():
    """10^6 distinct list keys emitted and dropped one after another (a
    long-running host worker): the intern table does not keep them (reference
    weak buckets, tuple.lua:250-302)."""
    import gc
    from lua_mapreduce_1_amd.utils.tuple import _INTERN, tuple as T
    base = len(_INTERN)
    peak = 0
    for i in range(1_000_000):
        k = T([i, "w", [i % 7]])
        assert k == (i, "w", (i % 7,))
        if i % 100_000 == 0:
            peak = max(peak, len(_INTERN))
    del k
    gc.collect()
    from lua_mapreduce_1_amd.utils.tuple import PRUNE_MIN
    assert peak <= base + 2 * PRUNE_MIN + 16
    assert T.stats()[0] <= base + 8
    keep = [T([i, [i]]) for i in range(3 * PRUNE_MIN)]  # live keys survive pruning
    assert all(T([i, [i]]) is keep[i] for i in range(0, len(keep), 997))
