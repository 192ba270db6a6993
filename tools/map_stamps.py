#!/usr/bin/env python
"""Where a word-count map wave's time goes: the map kernel
(csrc/hip/wordcount3.hip) instantiated with per-wave phase stamps over the
HBM-resident benchmark corpus, warm table.  Each wave reports its wall-clock
ticks in: the tile's five workgroup barriers (waiting for the slowest wave),
staging, start masks + scan, the token list, the token loop (LDS hash
inserts), and the flush to the HBM table.  Prints one JSON line: totals as
shares of the waves' time, the token loop's imbalance across the waves of a
workgroup, and the plain kernel's time for reference (the stamped
instantiation is timed too: its overhead is the difference).

    python tools/map_stamps.py [--cap-log2 23] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cap-log2", type=int, default=23)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dyn", type=int, default=None, help="DYN token lists on/off (default: MR_MAP_DYN)")
    a = ap.parse_args()
    import bench
    from lua_mapreduce_1_amd import ops
    from lua_mapreduce_1_amd.ops import _hip
    d = torch.device("cuda", 0)
    splits = bench.load_corpus()
    blob = b"".join(splits)
    text = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(d)
    n = text.numel()
    tab = ops.HashTable(1 << a.cap_log2, device=d, op="sum")
    lib = _hip.lib()
    if a.dyn is not None:
        lib.mr_wc3_set_dyn(a.dyn)
    f = lib.mr_wc_map3_stamped
    P, U64 = ctypes.c_void_p, ctypes.c_uint64
    f.argtypes = [P, U64, U64, P, P, P, U64, P, P, P, U64, P, P, P]
    f.restype = ctypes.c_int
    waves = 512 // 64
    nblocks = (n + 8192 - 1) // 8192
    stamps = torch.zeros(nblocks * waves * 8, dtype=torch.int64, device=d)
    ovf, counter = tab._overflow(n)
    slots, _h, _l, val, _r, ctrl = tab._gtab()

    def run(stamped: bool) -> float:
        tab.reset()
        counter.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if stamped:
            rc = f(_hip.ptr(text), n, 0, slots, val, ctrl, tab.cap, _hip.ptr(ovf[0]), _hip.ptr(ovf[1]),
                   _hip.ptr(ovf[2]), ovf[0].numel(), _hip.ptr(counter), _hip.ptr(stamps), _hip.stream(d))
            assert rc == 0, rc
        else:
            tab.wordcount_map(text)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    run(False)  # warm: the table's slots, the kernels
    plain = sorted(run(False) for _ in range(a.reps))
    stamped = sorted(run(True) for _ in range(a.reps))
    got, ovf_ = tab.stats()
    s = stamps.view(nblocks, waves, 8).cpu().numpy().astype(np.float64)
    total, bar, stage, scan, lst, loop, flush = (s[:, :, k] for k in range(7))
    T = total.sum()
    other = T - (bar + stage + scan + lst + loop + flush).sum()
    loop_imb = (loop.max(1) - loop.mean(1)).sum() / max(loop.sum() / waves, 1.0)
    out = {
        "dyn": a.dyn, "bytes": n, "blocks": nblocks, "table_cap": tab.cap, "distinct": got, "overflow": ovf_,
        "map_ms_plain_min": plain[0], "map_ms_plain_median": plain[len(plain) // 2],
        "map_ms_stamped_min": stamped[0], "map_ms_stamped_median": stamped[len(stamped) // 2],
        "share_of_wave_time": {
            "barrier_wait": bar.sum() / T, "staging": stage.sum() / T, "masks_scan": scan.sum() / T,
            "token_list": lst.sum() / T, "token_loop": loop.sum() / T, "flush": flush.sum() / T,
            "other (LDS init, prefetch issue)": other / T},
        "token_loop_imbalance": {"mean_excess_of_slowest_wave_over_mean": loop_imb,
                                 "p50_slowest_over_mean": float(np.median(loop.max(1) / np.maximum(loop.mean(1), 1)))},
        "wave_ticks_mean": {"total": float(total.mean()), "barrier_wait": float(bar.mean()),
                            "token_loop": float(loop.mean()), "flush": float(flush.mean())},
        "note": "ticks of wall_clock64 (100 MHz); shares summed over every wave of the launch",
    }
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
