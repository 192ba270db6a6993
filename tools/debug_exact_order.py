#!/usr/bin/env python
"""Check of the tail's exact-order fallback (ops.exact_key_perm) on the
bigram keys of the Europarl-shaped corpus: the permutation must be a
bijection, sort the rows by (partition, key bytes), and keep the value sum;
compared with the host order of the same rows."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lua_mapreduce_1_amd import ops  # noqa: E402
from lua_mapreduce_1_amd.runtime import device as dv  # noqa: E402
from lua_mapreduce_1_amd.utils import corpus  # noqa: E402


def main():
    d = torch.device("cuda:0")
    nsplit = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    splits = corpus.europarl_like(seed=1234)[:nsplit]
    text = b"".join(splits)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(d)
    import importlib
    B = importlib.import_module("lua_mapreduce_1_amd.examples.Bigram")
    ctx = dv.DeviceMapContext(d, "sum", 1 << 24)
    B.device_mapfn(1, t, ctx.emit)
    n, ovf = ctx.table.stats()
    hi, lo, val, rep = ctx.table.compact((n, ovf))
    src = ctx.source()
    nparts = 10
    part = dv.partition_of(hi, lo, rep, src, nparts, None)
    perm = ops.exact_key_perm(part, hi, lo, rep, src, nparts)
    p = perm.cpu().numpy()
    print("rows", n, "bijection", np.array_equal(np.sort(p), np.arange(n)), flush=True)
    print("value sum", int(val.sum()), int(val[perm].sum()), flush=True)
    off, blob = ops.gather_key_bytes(hi[perm], lo[perm], rep[perm], src, capacity=max(src.numel(), 32 * n))
    o = off.cpu().numpy()
    b = blob.cpu().numpy().tobytes()
    pp = part[perm].cpu().numpy()
    keys = [b[o[i]:o[i + 1]] for i in range(n)]
    bad = sum(1 for i in range(1, n) if (pp[i - 1], keys[i - 1]) > (pp[i], keys[i]))
    print("out of order", bad, "distinct", len(set(keys)), flush=True)
    return 0 if bad == 0 else 3


if __name__ == "__main__":
    sys.exit(main())
