"""Pinned host -> HBM copy bandwidth (the bound of the staged map phase)."""
import torch
for mb in (4, 32, 292):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        d.copy_(h, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"H2D {mb:4d} MB: {ms:7.3f} ms  {n / ms / 1e6:6.1f} GB/s", flush=True)
