#!/usr/bin/env python
"""A/B of the record gather (csrc/hip/records.hip) on TeraSort's 10 GB of
100-byte rows with a random permutation: the production word-per-lane
gather (mr_rec_gather: 25 lanes per row, 8 words in flight per thread)
against the row-per-lane candidate (mr_rec_gather_rows: 7 aligned 16-byte
loads per row, LDS slab, coalesced 16-byte stores).  Both outputs must be
identical.  Prints min/median ms of each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd.ops import _hip  # noqa: E402


def main():
    d = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    rb = 100
    rec = torch.randint(0, 256, (n * rb,), dtype=torch.uint8, device=d)
    perm = torch.randperm(n, device=d, dtype=torch.int64).to(torch.int32)
    s = _hip.stream(d)
    outs = {}
    for name in ("mr_rec_gather", "mr_rec_gather_rows"):
        out = torch.empty(n * rb, dtype=torch.uint8, device=d)
        ts = []
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _hip.call(name, _hip.ptr(rec), _hip.ptr(perm), n, rb, _hip.ptr(out), s)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        outs[name] = out
        print(f"{name:20s} min {ts[0]:.3f} ms  median {ts[len(ts) // 2]:.3f} ms  ({2 * n * rb / ts[0] / 1e9:.2f} TB/s)",
              flush=True)
    ok = torch.equal(outs["mr_rec_gather"], outs["mr_rec_gather_rows"])
    print("identical:", ok)
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
