"""Where the cold first iteration's time goes on the host: pinned allocation
of the rank's split buffer (torch caching host allocator, first and second
time), and the native loader reading the split files with the page cache
dropped into pinned (exact size, mr_host_alloc, or torch's power-of-two pool) vs pageable memory,
with 8 / 16 / 32 reader threads.  Usage: python tools/cold_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import corpus_dir, ensure_corpus  # noqa: E402
from lua_mapreduce_1_amd.ops import io as mio  # noqa: E402
from lua_mapreduce_1_amd.utils import corpus  # noqa: E402

torch.zeros(1, device="cuda")
d = corpus_dir(1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
ensure_corpus(d, 1234, corpus.EUROPARL_LINES, corpus.EUROPARL_WORDS)
paths = sorted(os.path.join(d, "files", f) for f in os.listdir(os.path.join(d, "files")))
lens = np.array([os.path.getsize(p) for p in paths], dtype=np.int64)
n = int(lens.sum() + len(paths))
for label, pin, threads in (("exact pinned", "exact", 8), ("torch pinned", True, 8), ("torch pinned again", True, 8),
                            ("exact pinned 16 thr", "exact", 16), ("exact pinned 32 thr", "exact", 32),
                            ("pageable", False, 8)):
    t0 = time.perf_counter()
    buf = mio.pinned_empty(n) if pin == "exact" else torch.empty(n, dtype=torch.uint8, pin_memory=pin)
    t1 = time.perf_counter()
    for p in paths:
        mio.drop_page_cache(p)
    off = np.zeros(len(paths), dtype=np.int64)
    np.cumsum(lens[:-1] + 1, out=off[1:])
    t2 = time.perf_counter()
    ld = mio.AsyncLoad(paths, np.zeros(len(paths), dtype=np.int64), lens, off, np.ones(len(paths), dtype=np.int64),
                       buf, threads=threads)
    ld.wait()
    t3 = time.perf_counter()
    print(f"{label:20s} alloc {1e3 * (t1 - t0):7.2f} ms  read {n / 1e6:.0f} MB cold {1e3 * (t3 - t2):7.2f} ms "
          f"({n / (t3 - t2) / 1e9:.2f} GB/s)", flush=True)
    if not pin:
        del buf
