"""The per-module unit tests run through the aggregator (reference:
mapreduce/test.lua, which test.sh runs first)."""
from lua_mapreduce_1_amd import test as agg


def test_module_utests():
    agg.run()
