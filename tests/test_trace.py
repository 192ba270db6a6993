"""roctx phase ranges (utils/trace.py): off by default, and when enabled the
push/pop/mark calls go through the ROCm tracing library without a profiler
attached (no-ops there) and an SPMD iteration still runs."""
from lua_mapreduce_1_amd.utils import trace


def test_trace_disabled_by_default_and_nestable():
    with trace.range("outer"):
        with trace.range("inner"):
            trace.mark("m")


def test_trace_enabled_ranges_run():
    was = trace.enabled()
    try:
        avail = trace.enable(True)
        with trace.range("mr.test"):
            trace.mark("mr.test.mark")
        # the library is part of every ROCm install; without it ranges are no-ops
        assert avail in (True, False)
    finally:
        trace.enable(was)


def test_spmd_iteration_with_ranges_on_cpu():
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    M = "lua_mapreduce_1_amd.models.wordcount"
    splits = europarl_like(seed=4, lines=2000, words=20_000, vocab_size=2_000, split_lines=500)
    was = trace.enabled()
    trace.enable(True)
    try:
        eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                              init_args={"nsplits": len(splits), "num_reducers": 3}),
                         split_store=SplitStore(splits, pin=False), device="cpu")
        res = eng.run_iteration()
        assert res.total_value == 20_000
    finally:
        trace.enable(was)
