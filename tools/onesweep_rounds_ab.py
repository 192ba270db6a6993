"""Onesweep tile size A/B (csrc/hip/sort.hip, MR_SORT_ROUNDS = keys per
thread of the tiles of sorts of >= 4 M keys, 256 threads per tile): TeraSort's sort (100 M random u64 keys, top 32
bits, int32 permutation: 4 passes) and a keys-only sort of 46 M keys (3
passes, the inverted index's shape), min / median of 7; outputs checked
against torch.sort.  Usage: python tools/onesweep_rounds_ab.py [rounds ...]"""
import sys
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import _hip

g = torch.Generator(device="cuda").manual_seed(0)
hi = torch.randint(-2**63, 2**63 - 1, (100_000_000,), dtype=torch.int64, device="cuda", generator=g)
ko = torch.randint(0, 1 << 24, (46_000_000,), dtype=torch.int64, device="cuda", generator=g)
sign = -(1 << 63)
ref_top = torch.sort((hi >> 32) & 0xFFFFFFFF, stable=True).values
ref_ko = torch.sort(ko).values


def timed(fn):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[0], ts[len(ts) // 2]


for r in [int(x) for x in sys.argv[1:]] or [16, 24, 32]:
    assert _hip.lib().mr_sort_set_rounds(r) == 0
    mn, md = timed(lambda: ops.sort_keys([hi], bits=[64], return_keys=True, from_bit=32))
    perm, sk = ops.sort_keys([hi], bits=[64], return_keys=True, from_bit=32)
    ok1 = torch.equal((sk >> 32) & 0xFFFFFFFF, ref_top) and torch.equal(hi[perm.long()], sk)
    mn2, md2 = timed(lambda: ops.sort_keys([ko], bits=[24], keys_only=True))
    _, sko = ops.sort_keys([ko], bits=[24], keys_only=True)
    ok2 = torch.equal(sko, ref_ko)
    print(f"rounds {r:2d}: top32+perm 100M min {mn:6.3f} med {md:6.3f} ms ({mn / 4:5.3f}/pass) ok={ok1} | "
          f"keys-only 24-bit 46M min {mn2:6.3f} med {md2:6.3f} ms ok={ok2} err={ops.sort_error(hi.device)}",
          flush=True)
