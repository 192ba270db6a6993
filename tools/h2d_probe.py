"""Host->HBM bandwidth of the ways to stage a rank's input (36 MB = 1/8 of
the corpus, 291 MB = all of it): one SDMA hipMemcpyAsync, the same split over
two streams (two engines?), and shader loads from pinned host memory
(mr_h2d_pull) at several grid sizes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402

_hip.lib()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
p1, p2 = _hip.stream_ptr(s1), _hip.stream_ptr(s2)


def timed(fn, reps=6):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        e0.record(s1)
        s2.wait_event(e0)
        fn()
        ev = torch.cuda.Event()
        ev.record(s2)
        s1.wait_event(ev)
        e1.record(s1)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


for mb in (36, 291):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.fill_(3)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    res["sdma x1"] = timed(lambda: _hip.call("mr_memcpy_async", _hip.ptr(d), _hip.ptr(h), n, 1, p1))
    half = (n // 2) & ~4095

    def two():
        _hip.call("mr_memcpy_async", _hip.ptr(d), _hip.ptr(h), half, 1, p1)
        _hip.call("mr_memcpy_async", _hip.ptr(d[half:]), _hip.ptr(h[half:]), n - half, 1, p2)
    res["sdma x2 streams"] = timed(two)
    for blocks in (256, 1024, 4096):
        res[f"pull {blocks} WGs"] = timed(lambda: _hip.call("mr_h2d_pull", _hip.ptr(d), _hip.ptr(h), n, blocks, p1))
    assert bool((d[:4096] == 3).all()) and bool((d[-4096:] == 3).all())
    for k, ms in res.items():
        print(f"{mb:4d} MB  {k:18s} {ms:7.3f} ms  {n / ms / 1e6:6.1f} GB/s", flush=True)
