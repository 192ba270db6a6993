"""Large result downloads on the SDMA copy engines (csrc/hip/sdma.hip,
runtime/device.py dma_to_host / flush_downloads) against torch's own copy."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sdma_downloads_match():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lua_mapreduce_1_amd.ops import _hip
    from lua_mapreduce_1_amd.runtime import device as dv
    assert _hip.lib().mr_sdma_available() == 1
    d = torch.device("cuda", 0)
    srcs = [torch.randint(0, 2**62, (n,), dtype=torch.int64, device=d) for n in (3 << 20, 5 << 20, 17)]
    dsts = [torch.empty(s.numel(), dtype=torch.int64, pin_memory=True) for s in srcs]
    for h, s in zip(dsts, srcs):
        dv.dma_to_host(h, s)
    assert len(dv._SDMA.get(d, [])) == 2  # the two >= 8 MiB downloads are deferred, the small one is not
    _hip.wait_stream(d)
    dv.flush_downloads(d)
    assert dv._SDMA["ok"] is True
    for h, s in zip(dsts, srcs):
        assert torch.equal(h, s.cpu())


def test_small_reads_one_launch():
    """host_read_begin: small tensors of several dtypes (and an odd byte
    count) downloaded by one launch that signals the host; the host work
    between begin and wait overlaps it; a later signal on the stream does not
    hide an earlier one."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lua_mapreduce_1_amd import ops
    from lua_mapreduce_1_amd.ops import _hip
    d = torch.device("cuda", 0)
    ts = [torch.arange(24, dtype=torch.int64, device=d).view(8, 3), torch.tensor([7, -1], dtype=torch.int32, device=d),
          torch.arange(5, dtype=torch.uint8, device=d), torch.tensor([1.5], dtype=torch.float64, device=d)]
    w0 = _hip.WAITS[0]
    rd = ops.host_read_begin(ts)
    assert rd.sig is not None
    x = torch.ones(1 << 20, device=d) * 3  # more work queued behind it, then another signal on the stream
    _hip.wait_stream(d)
    got = rd.wait()
    for a, t in zip(got, ts):
        assert a.shape == tuple(t.shape) and (a == t.cpu().numpy()).all()
    assert _hip.WAITS[0] - w0 == 2 and float(x[0]) == 3.0
    assert ops.host_read_begin([torch.zeros(1 << 17, dtype=torch.int64, device=d)]).sig is None  # large: blits


def test_signal_order_helper():
    from lua_mapreduce_1_amd.ops import _hip
    assert _hip._done(5, 5) and _hip._done(6, 5) and not _hip._done(4, 5) and not _hip._done(0, 5)
    assert _hip._done(2, 0x7FFFFFFF)  # wrapped


def test_lazy_batch_lands_and_guards_buffers():
    """flush_downloads(wait=False): the batch is in flight when it returns,
    its bytes are in place after wait(); a small stream copy into a buffer
    the batch fills waits for it first (the batch must not land over it)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lua_mapreduce_1_amd.ops import _hip
    from lua_mapreduce_1_amd.runtime import device as dv
    d = torch.device("cuda", 0)
    src = torch.randint(0, 2**62, (9 << 20,), dtype=torch.int64, device=d)
    dst = torch.empty(src.numel(), dtype=torch.int64, pin_memory=True)
    dv.dma_to_host(dst, src)
    _hip.wait_stream(d)
    b = dv.flush_downloads(d, wait=False)
    assert b is not None and not b.done and dv._INFLIGHT.get(d) is b
    assert b.writes(dst.data_ptr() + 8, 16) and not b.writes(dst.data_ptr() + dst.numel() * 8, 8)
    small = torch.full((4,), -7, dtype=torch.int64, device=d)
    dv.dma_to_host(dst[:4], small)  # overlaps the batch: waits for it, then copies on the stream
    assert b.done and d not in dv._INFLIGHT
    _hip.wait_stream(d)
    assert dst[:4].tolist() == [-7] * 4 and torch.equal(dst[4:], src[4:].cpu())
    b2 = None
    dv.dma_to_host(dst, src)
    _hip.wait_stream(d)
    b2 = dv.flush_downloads(d, wait=False)
    dv.wait_downloads()
    assert b2.done and torch.equal(dst, src.cpu())


def test_lazy_exact_tail_results(monkeypatch):
    """The exact-order tail (n-gram keys) returns its iteration's results
    while their download is still landing; reading them waits.  Three
    pipelined iterations, each checked against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import dataclasses
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_generic_plane import BG, close_lists, make_data, oracle
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils import config
    monkeypatch.setattr(config, "TUNABLES", dataclasses.replace(config.TUNABLES, sdma_min_mb=1e-4))
    d = torch.device("cuda", 0)
    splits = make_data("text")
    exp = oracle("text", "bigram", splits)
    eng = SPMDEngine(dict(taskfn=BG, mapfn=BG, partitionfn=BG, reducefn=BG, finalfn=None,
                          init_args={"mode": "bigram", "nsplits": len(splits)}),
                     split_store=SplitStore(splits, pin=True), device=d)
    eng.prefetch, eng.pipeline = True, True
    eng._exact_tail = True  # the order a long n-gram run falls back to, from the first iteration
    steps, lazy = 3, 0
    for k in range(steps):
        res = eng.run_iteration(prefetch_next=k < steps - 1, lookahead=steps - 1 - k)
        lazy += getattr(res, "_dl", None) is not None
        got = {}
        for _n, cols in eng.gather_results(res):
            for key, v in codec.iter_columnar(cols):
                got[key] = list(v)
        assert close_lists(got, exp), k
        assert res.distinct_keys == len(exp)
    # the first tail can grow past the key-byte estimate a previous engine
    # left (a top-up copy, eager); the later ones stay in flight
    assert lazy >= steps - 1
