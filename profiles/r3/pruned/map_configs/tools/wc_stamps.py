"""Per-workgroup phase timestamps of the v3 word-count map kernel:
start -> end of tile loop (clear + tokenize + LDS combine) -> end of flush."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.utils.corpus import europarl_like

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 0
chunk = {0: 8192, 1: 16384, 2: 16384, 3: 4096, 4: 8192, 5: 16384}[cfg]
text = b"".join(europarl_like())
dev = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
tab = ops.HashTable(1 << 21, device="cuda")
for frac, name in ((1, "full"), (8, "1/8")):
    data = dev[: len(text) // frac]
    nwg = (data.numel() + chunk - 1) // chunk
    st = torch.zeros(4 * nwg, dtype=torch.int64, device="cuda")
    for _ in range(3):
        tab.reset()
        tab.wordcount_map(data, mode=cfg, stamps=st)
    torch.cuda.synchronize()
    s = st.view(-1, 4).cpu().numpy()
    t0 = s[:, 0].min()
    a, b, c = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0, (s[:, 2] - t0) / 100.0  # 100 MHz -> us
    print(f"{name}: cfg{cfg} {nwg} workgroups, span {c.max():.1f} us")
    print(f"  per-WG loop (clear+tokenize+LDS) us: median {np.median(b - a):.2f} p90 {np.percentile(b - a, 90):.2f}"
          f"  flush us: median {np.median(c - b):.2f} p90 {np.percentile(c - b, 90):.2f} max {np.max(c - b):.2f}")
    xcc = (s[:, 3] >> 32) & 0xF
    for q in (0.1, 0.5, 0.9, 1.0):
        print(f"  {int(q*100):3d}% of WGs started by {np.quantile(a, q):8.1f} us, ended by {np.quantile(c, q):8.1f} us")
    ends = [c[xcc == x].max() if (xcc == x).any() else 0 for x in range(8)]
    print("  per-XCD end us:", [round(float(e), 1) for e in ends])
