#!/usr/bin/env python
"""A/B of the record key pass (csrc/hip/records.hip): the tiled kernel
(coalesced 16-byte loads of 256 whole rows into LDS) against the per-row
strided 4-byte loads, on TeraSort's 10 GB of 100-byte rows; both must give
the same keys and histograms.  Prints min/median ms of each."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402


def main():
    d = torch.device("cuda:0")
    n, rb, kb = 100_000_000, 100, 10
    rec = torch.randint(0, 256, (n * rb,), dtype=torch.uint8, device=d)
    s = _hip.stream(d)
    out = {}
    for name in ("mr_rec_keys32", "mr_rec_keys32_strided"):
        k32 = torch.empty(n, dtype=torch.int32, device=d)
        gh = torch.zeros(2048, dtype=torch.int32, device=d)
        ts = []
        for _ in range(8):
            gh.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _hip.call(name, _hip.ptr(rec), n, rb, kb, _hip.ptr(k32), _hip.ptr(gh), s)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        out[name] = (k32.clone(), gh.clone())
        print(f"{name:24s} min {ts[0]:.3f} ms  median {ts[len(ts) // 2]:.3f} ms  ({n * rb / ts[0] / 1e9:.2f} TB/s of rows)",
              flush=True)
    a, b = out["mr_rec_keys32"], out["mr_rec_keys32_strided"]
    ok = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    print("same keys and histograms:", ok)
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
