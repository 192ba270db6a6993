"""TeraSort key pass with and without the fused digit histograms (10 GB of
100-byte rows): is the pass bound by its LDS histogram atomics or by its
row reads?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lua_mapreduce_1_amd.ops import records as RC  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    d = torch.device("cuda", 0)
    n, rb = 100_000_000, 100
    rec = torch.randint(0, 256, (n, rb), dtype=torch.uint8, device=d)
    gh = torch.zeros(2048, dtype=torch.int32, device=d)
    print("keys32 + ghist   %.3f ms" % timed(lambda: (gh.zero_(), RC.keys32(rec, 10, gh))))
    print("keys32 no ghist  %.3f ms" % timed(lambda: RC.keys32(rec, 10, None)))
    k = RC.keys32(rec, 10, None)
    print("k32 sum (u32 view as u64 ghist input proxy) ok", int(k.numel()))


if __name__ == "__main__":
    main()
