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
