"""Combiner and batched reducers on the GPU: the segmented-fold kernel
(csrc/hip/segments.hip) against NumPy, the general plane's combiner modes on
cuda:0, and a hot key of more than 10 M values within a time and an HBM
bound (the batched MAX_MAP_RESULT of /root/reference/mapreduce/job.lua:92-96)."""
import os
import sys
import time

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_combiner import CM, _oracle, _rand_csr  # noqa: E402
from test_generic_plane import close_lists, make_data, run_engine  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,hot", [(0, 5000), (1, 3_000_000), (2, 1)])
@pytest.mark.parametrize("dtype", ["i64", "f64"])
def test_seg_reduce_kernel_matches_numpy(gpu, seed, hot, dtype):
    from lua_mapreduce_1_amd.ops import segments as S
    off, val = _rand_csr(seed, m=20_000, hot=hot)
    if dtype == "f64":
        val = val.astype(np.float64) / 3.0
    o, v = torch.from_numpy(off).to(gpu), torch.from_numpy(val).to(gpu)
    for op in ("sum", "min", "max"):
        got = S.reduce(o, v, op).cpu().numpy()
        exp = S.reduce(torch.from_numpy(off), torch.from_numpy(val), op).numpy()
        if dtype == "f64" and op == "sum":
            assert np.allclose(got, exp, rtol=1e-9, atol=1e-6), op
        else:
            assert np.array_equal(got, exp), op


def test_seg_helpers_gpu_match_cpu(gpu):
    from lua_mapreduce_1_amd.ops import segments as S
    off, val = _rand_csr(4, m=5000, hot=20_000)
    oc, vc = torch.from_numpy(off), torch.from_numpy(val)
    og, vg = oc.to(gpu), vc.to(gpu)
    for f in (lambda o, v: S.topk(o, v, 4), S.unique):
        a, b = f(oc, vc), f(og, vg)
        assert torch.equal(a[0], b[0].cpu()) and torch.equal(a[1], b[1].cpu())
    assert torch.equal(S.nunique(oc, vc), S.nunique(og, vg).cpu())
    assert torch.allclose(S.median(oc, vc), S.median(og, vg).cpu(), equal_nan=True)


@pytest.mark.parametrize("mode", ["host", "device", "topk", "median"])
def test_combiner_modes_gpu(gpu, mode):
    import comb_modules
    splits = make_data("text")
    comb_modules.CALLS.update(combinerfn=0, reducefn=0)
    eng, res, got = run_engine(CM, splits, gpu, {"mode": mode})
    assert close_lists(got, _oracle(splits, mode))
    if mode != "median":
        assert eng.plane.map.combines == 1
    if mode in ("device", "topk", "median"):
        assert comb_modules.CALLS["reducefn"] == 0


@pytest.mark.parametrize("hot_device", [True, False], ids=["device_combiner", "host_combiner"])
def test_hot_key_12m_values_gpu(gpu, hot_device):
    """4 splits x 3 M values of one key = 12 M values: combined every 2^22
    postings, the job stays under 1.5 GiB of extra HBM and finishes in
    seconds (the host combiner sums 12 M Python ints)."""
    splits = make_data("text")
    hot = 3_000_000
    run_engine(CM, splits[:1], gpu, {"mode": "hot", "hot": 1000, "hot_device": hot_device})  # warm-up
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    t0 = time.time()
    eng, res, got = run_engine(CM, splits, gpu, {"mode": "hot", "hot": hot, "hot_device": hot_device},
                               combine_postings=1 << 22)
    dt = time.time() - t0
    peak = torch.cuda.max_memory_allocated() - base
    assert close_lists(got, _oracle(splits, "hot", hot))
    assert eng.plane.map.combines >= 2
    assert peak < 1.5 * (1 << 30), peak
    assert dt < (20 if hot_device else 60), dt
