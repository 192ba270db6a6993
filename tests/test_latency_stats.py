"""examples/LatencyStats: percentiles per key through device_reducefn (no
combiner, float64 value lists) against the per-key Python reducer, on the
CPU engine and on the GPU."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_generic_plane import close_lists, run_engine  # noqa: E402

M = "lua_mapreduce_1_amd.examples.LatencyStats"


def _check(device):
    import importlib
    mod = importlib.import_module(M)
    splits = mod.make_log(seed=4, lines=30_000, endpoints=150)
    eng, res, got = run_engine(M, splits, device, {"num_reducers": 5})
    want = mod.naive(splits)
    assert len(want) > 50
    assert close_lists(got, want, rel=1e-12)
    assert res.failed_maps == 0


def test_latency_stats_cpu():
    _check(torch.device("cpu"))


@pytest.mark.gpu
def test_latency_stats_gpu(gpu):
    _check(gpu)
