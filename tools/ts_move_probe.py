"""TeraSort data movement on one MI355X: copy / random-row gather / random-row
scatter / gather inside windows (what an MSD bucket pass would leave) of
100-byte rows, 100 M rows = 10 GB (tools/probe/ts_move.hip).  Decides whether
a bucketing pass can pay for itself (profiles/r3/terasort/).
Usage: python tools/ts_move_probe.py [n_rows]"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "probe", "libtsmove.so")
if not os.path.exists(SO):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(HERE, "probe", "ts_move.hip"), "-o", SO])
L = ctypes.CDLL(SO)
for f in ("probe_copy",):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
L.probe_bucket.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
for f in ("probe_gather", "probe_scatter"):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
dev = torch.device("cuda")
rec = torch.randint(0, 1 << 30, (n * 25,), dtype=torch.int32, device=dev)
out = torch.empty_like(rec)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


gb = n * 100 / 1e9
t = timeit(lambda: L.probe_copy(P(rec), P(out), n * 100, s))
print(f"copy       {t:7.3f} ms  {2 * gb / t:6.2f} TB/s (read+write)", flush=True)
perm = torch.randperm(n, device=dev, dtype=torch.int64).to(torch.int32)
t = timeit(lambda: L.probe_gather(P(rec), P(perm), n, P(out), s))
print(f"gather     {t:7.3f} ms  {2 * gb / t:6.2f} TB/s", flush=True)
inv = torch.empty_like(perm)
inv[perm.long()] = torch.arange(n, device=dev, dtype=torch.int32)
t = timeit(lambda: L.probe_scatter(P(rec), P(inv), n, P(out), s))
print(f"scatter    {t:7.3f} ms  {2 * gb / t:6.2f} TB/s", flush=True)
for win_mb in (8, 40, 160):
    win = win_mb * 10_000
    base = torch.arange(n, device=dev, dtype=torch.int64) // win * win
    r = torch.rand(n, device=dev)
    order = torch.argsort(base.double() + r)  # random inside each window
    pw = order.to(torch.int32)
    del base, r, order
    t = timeit(lambda: L.probe_gather(P(rec), P(pw), n, P(out), s))
    print(f"gather_w{win_mb:<4d}{t:7.3f} ms  {2 * gb / t:6.2f} TB/s (perm random inside {win_mb} MB windows)",
          flush=True)

# MSD bucket pass: rows into 2^b bucket regions of capacity n/2^b * 1.05
del perm, inv
for bbits in (4, 6, 8):
    nb = 1 << bbits
    bcap = int(n / nb * 1.05) + 4096
    big = torch.empty(nb * bcap * 25, dtype=torch.int32, device=dev)
    keys = torch.empty(nb * bcap, dtype=torch.int32, device=dev)
    cur = torch.zeros(nb, dtype=torch.int64, device=dev)

    def run():
        cur.zero_()
        L.probe_bucket(P(rec), n, bbits, bcap, P(cur), P(big), P(keys), s)
    t = timeit(run)
    ok = int(cur.sum()) == n and int(cur.max()) <= bcap
    print(f"bucket{nb:<5d}{t:7.3f} ms  {2 * gb / t:6.2f} TB/s (rows read in order, written to {nb} bucket "
          f"regions, + keys) {'ok' if ok else 'OVERFLOW'}", flush=True)
    del big, keys
