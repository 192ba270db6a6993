"""Row gather of 10 GB of 100-byte rows by a random permutation: the
pipelined 16-byte LDS gather (next batch's loads issued before the current
batch's stores, the default) against the unpipelined form (mode 2)."""
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
    perm = torch.randperm(n, device=d).to(torch.int32)
    a = RC.gather(rec, perm, mode=0)
    b = RC.gather(rec, perm, mode=2)
    print("equal", bool(torch.equal(a, b)), bool(torch.equal(a[:1000], rec[perm[:1000].long()])))
    del a, b
    for rep in range(2):
        print("pipelined   %.3f ms" % timed(lambda: RC.gather(rec, perm, mode=0)))
        print("unpipelined %.3f ms" % timed(lambda: RC.gather(rec, perm, mode=2)))


if __name__ == "__main__":
    main()
