"""Reduce rounds (reduce_cap_mb) on the GPU: inverted index on the list and
general planes, value-list reducers (host and batched device) and typed
folds, against their oracles (CPU variants: test_reduce_rounds.py)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_generic_plane import SS, close_lists, make_data, oracle, run_engine  # noqa: E402
from test_reduce_rounds import CAP, _inv_index  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("plane", ["list", "generic"])
def test_inverted_index_in_reduce_rounds_gpu(gpu, plane):
    extra = {"plane": "generic"} if plane == "generic" else {}
    eng, res, got, exp = _inv_index(gpu, reduce_cap_mb=CAP, table_capacity=1 << 16, **extra)
    assert eng.plane_kind == plane and eng.plane.reduce_rounds > 2
    assert got == exp


@pytest.mark.parametrize("mode", ["host", "device", "topk", "median"])
def test_value_list_reducers_in_reduce_rounds_gpu(gpu, mode):
    import comb_modules
    splits = make_data("text")
    eng, res, got = run_engine("comb_modules", splits, gpu, {"mode": mode}, reduce_cap_mb=CAP)
    assert eng.plane.reduce_rounds > 2
    assert close_lists(got, comb_modules.oracle(splits, mode))


def test_typed_folds_in_reduce_rounds_gpu(gpu):
    splits = make_data("scores")
    eng, res, got = run_engine(SS, splits, gpu, {}, reduce_cap_mb=CAP)
    assert eng.plane.reduce_rounds > 2
    assert close_lists(got, oracle("scores", None, splits))
