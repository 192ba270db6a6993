"""Host time of each hipMemcpyAsync (pinned -> HBM) in a fresh process: which
call stalls, and does the copy engine choice matter (HSA_ENABLE_SDMA)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402

n = 37 << 20
host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
host.fill_(1)
dev = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2)]
cs = torch.cuda.Stream()
sp = _hip.stream_ptr(cs)
sizes = [2 << 20, 8 << 20, 17 << 20, 8 << 20, 2 << 20]
_hip.lib()
for it in range(12):
    off = 0
    line = []
    for sz in sizes:
        t = time.perf_counter()
        _hip.call("mr_memcpy_async", _hip.ptr(dev[it % 2][off:off + sz]), _hip.ptr(host[off:off + sz]), sz, 1, sp)
        line.append(1000 * (time.perf_counter() - t))
        off += sz
    t = time.perf_counter()
    cs.synchronize()
    print(f"iter {it}: issue ms {[round(x, 3) for x in line]}  sync {1000 * (time.perf_counter() - t):.3f}",
          flush=True)
