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
