"""Per-pass timing of the onesweep radix sort on n random u64 keys (+u32 perm)."""
import sys
import torch
import numpy as np
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
k = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda")
for bits in (8, 64):
    ops.sort_keys([k], bits=[bits])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        ops.sort_keys([k], bits=[bits])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"n={n} bits={bits}: {ms:.3f} ms, {ms / (bits // 8):.3f} ms/pass, "
          f"{n * 24 / (ms / (bits // 8)) / 1e9:.0f} GB/s per pass (key+idx in/out)", flush=True)
