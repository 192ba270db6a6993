"""Does a small device->host download on the compute stream wait behind large
host->device copies queued earlier on ANOTHER stream (shared SDMA engine)?

Queues `--ahead` x 36 MB H2D copies on a copy stream, then on the compute
stream a tiny kernel followed by a 1 MB D2H, either by hipMemcpyAsync (SDMA)
or by the copy_to_host kernel (shader stores over PCIe).  Prints when the D2H
completes relative to the start, next to the H2D completion time.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402

N = 36 << 20
M = 1 << 20
host = [torch.empty(N, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
for h in host:
    h.fill_(1)
dev = [torch.empty(N, dtype=torch.uint8, device="cuda") for _ in range(3)]
small = torch.ones(M, dtype=torch.uint8, device="cuda")
hsmall = torch.empty(M, dtype=torch.uint8, pin_memory=True)
nel = torch.tensor([M], dtype=torch.int64, device="cuda")
cs = torch.cuda.Stream()
ms = torch.cuda.current_stream()
csp, msp = _hip.stream_ptr(cs), _hip.stream_ptr(ms)
_hip.lib()


def once(mode: str, ahead: int):
    torch.cuda.synchronize()
    e_copy = torch.cuda.Event(enable_timing=True)
    e_d2h = torch.cuda.Event(enable_timing=True)
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record(ms)
    cs.wait_event(t0)
    for k in range(ahead):
        _hip.call("mr_memcpy_async", _hip.ptr(dev[k]), _hip.ptr(host[k]), N, 1, csp)
    e_copy.record(cs)
    small.add_(1)
    if mode == "sdma":
        _hip.call("mr_memcpy_async", _hip.ptr(hsmall), _hip.ptr(small), M, 2, msp)
    else:
        _hip.call("mr_copy_to_host", _hip.ptr(small), _hip.ptr(hsmall), _hip.ptr(nel), 1, M, msp)
    e_d2h.record(ms)
    torch.cuda.synchronize()
    return t0.elapsed_time(e_copy), t0.elapsed_time(e_d2h)


for mode in ("sdma", "kernel"):
    for ahead in (0, 1, 3):
        r = [once(mode, ahead) for _ in range(6)][2:]
        c = sorted(x[0] for x in r)[len(r) // 2]
        d = sorted(x[1] for x in r)[len(r) // 2]
        print(f"{mode:6s} ahead={ahead}: H2D done {c:7.3f} ms   D2H done {d:7.3f} ms", flush=True)
