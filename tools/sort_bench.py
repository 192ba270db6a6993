"""Onesweep radix sort (csrc/hip/sort.hip) of 136-bit keys (8 + 64 + 64 bits:
the reduce side's (partition, key) shape) at several sizes: ms per sort and
keys/s.  Usage: python tools/sort_bench.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops  # noqa: E402

for n in (300_000, 2_000_000, 12_500_000):
    rng = np.random.default_rng(0)
    w = [torch.from_numpy(rng.integers(0, 10, n).astype(np.int64)).cuda(),
         torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)).cuda(),
         torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)).cuda()]
    ops.sort_keys(w, [8, 64, 64])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.sort_keys(w, [8, 64, 64])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"n={n:>9} onesweep {ms:8.3f} ms  {n / ms / 1e3:8.1f} Mkeys/s (136-bit keys)", flush=True)
