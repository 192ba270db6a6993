"""TeraSort row gather (100-byte records, random permutation) — variants of
mr_ts_gather_mode at 100 M records (10 GB in, 10 GB out)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
rec = torch.randint(0, 1 << 30, (n * 25,), dtype=torch.int32, device="cuda")
perm = torch.randperm(n, device="cuda", dtype=torch.int64).to(torch.int32)
out = torch.empty_like(rec)
ref = None
for mode, grid in [(0, 0), (1, 0), (2, 0), (3, 0), (4, 0), (2, 4096), (2, 16384), (4, 4096), (4, 16384)]:
    def run():
        _hip.call("mr_ts_gather_mode", _hip.ptr(rec), _hip.ptr(perm), n, _hip.ptr(out), mode, grid,
                  _hip.stream())
    run()
    torch.cuda.synchronize()
    chk = int(out[::9973].sum())
    if ref is None:
        ref = chk
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(4):
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    print(f"mode {mode} grid {grid:6d}: {best:7.3f} ms  {2 * n * 100 / best / 1e9:6.2f} TB/s (in+out)  "
          f"{'ok' if chk == ref else 'MISMATCH'}", flush=True)
