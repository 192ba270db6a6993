"""TeraSort-style distributed sort of 100-byte records (BASELINE.json config
"TeraSort-style 10 GB key/value sort on 8xMI355X (radix sort + all-to-all)").

As a MapReduce job this is identity map + range partitioner + identity
reduce with the framework's shuffle and per-partition key sort doing all the
work (the reference's partition / sort / k-way-merge path, SURVEY.md §2.2
K6/K7/K9/C1).  MI355X pipeline, one rank per GPU, data resident in HBM:

  1. (W > 1) splitters: every rank samples ``oversample * W`` key prefixes, one
     all-gather, sort, take W-1 evenly spaced — TeraSort's sampled total-order
     partitioner;
  2. (W > 1) destination per record (binary search over the splitters in LDS),
     one 8-bit radix pass orders the rows by destination, a row gather packs
     them contiguously, and ONE ``all_to_all_single`` moves the 100-byte rows
     (RCCL over xGMI; all 7 links at once);
  3. local LSD radix sort of the 64-bit key prefixes (onesweep, 8 passes over
     (key, index) pairs — the 100-byte rows are not moved per pass), a fix-up
     kernel ordering the rare equal-prefix runs by the last 2 key bytes, and one
     final row gather.

Rank r's output holds keys in [splitter r-1, splitter r); concatenated in
rank order the output is globally sorted.  ``validate`` checks order within and
across ranks and an order-independent checksum of all records.
"""
from __future__ import annotations

import time

import torch

from .. import ops
from ..ops import terasort as TS
from . import dist as D


class TeraSort:
    def __init__(self, total_records: int, group=None, device=None, seed: int = 0x7E5A, oversample: int = 1024):
        self.group = group
        self.rank, self.world = D.world_info(group)
        self.device = torch.device(device if device is not None else "cpu")
        self.total = int(total_records)
        per = self.total // self.world
        self.first = per * self.rank
        self.n = per if self.rank < self.world - 1 else self.total - per * (self.world - 1)
        self.seed = seed
        self.oversample = oversample
        self.timings: dict[str, float] = {}

    def generate(self) -> torch.Tensor:
        return TS.generate(self.n, self.first, self.seed, self.device)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def splitters(self, hi: torch.Tensor) -> torch.Tensor:
        """W-1 unsigned splitters (int64 bit patterns) from a global sample."""
        W = self.world
        k = min(self.oversample * W, max(1, hi.numel()))
        g = torch.Generator().manual_seed(self.seed * 7919 + self.rank)
        idx = torch.randint(0, max(1, hi.numel()), (k,), generator=g).to(hi.device)
        samp = hi[idx] if hi.numel() else torch.zeros(k, dtype=torch.int64, device=hi.device)
        allv = D.all_gather_tensor(samp, self.group)
        # unsigned order of int64 bit patterns: flip the sign bit, sort signed
        flipped = allv ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=allv.device)
        srt = torch.sort(flipped).values ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=allv.device)
        m = srt.numel()
        pick = torch.tensor([(m * j) // W for j in range(1, W)], dtype=torch.int64, device=srt.device)
        return srt[pick].contiguous()

    def sort(self, rec: torch.Tensor) -> torch.Tensor:
        """Globally sort ``rec`` ([n, 100] uint8) across ranks -> this rank's
        sorted output block."""
        t0 = time.perf_counter()
        W = self.world
        t_part = t0
        if W > 1:
            hi, _ = TS.keys(rec)
            sp = self.splitters(hi)
            dest = TS.dest_of(hi, sp)
            perm = ops.sort_keys([dest.to(torch.int64)], bits=[max(8, (W - 1).bit_length())])
            packed = TS.gather(rec, perm)
            counts = ops.bincount(dest, W)
            recv = D.exchange_counts(counts, self.group)
            both = torch.cat([counts, recv]).cpu().tolist()
            t_part = time.perf_counter()
            rec = D.all_to_all_v(packed, both[:W], both[W:], self.group)
            del packed
        t_shuf = time.perf_counter()
        hi, lo = TS.keys(rec)
        perm = TS.sort_perm(hi, lo)
        out = TS.gather(rec, perm)
        self._sync()
        t1 = time.perf_counter()
        self.timings = {"partition": t_part - t0, "shuffle": t_shuf - t_part, "local_sort": t1 - t_shuf,
                        "total": t1 - t0}
        return out

    def validate(self, out: torch.Tensor, checksum_in: int) -> dict:
        """Global order + record checksum (collective)."""
        hi, lo = TS.keys(out)
        bad = TS.unsorted_pairs(hi, lo)
        n = out.shape[0]
        edge = torch.zeros(4, dtype=torch.int64)
        if n:
            edge[0], edge[1] = int(hi[0]), int(lo[0])
            edge[2], edge[3] = int(hi[-1]), int(lo[-1])
        edges = D.gather_objects((n, edge.tolist()), 0, self.group)
        cs = D.gather_objects(TS.checksum(out), 0, self.group)
        tot_bad = D.all_reduce_sum_int(bad, self.device, self.group)
        count = D.all_reduce_sum_int(n, self.device, self.group)
        res = {"unsorted_pairs": tot_bad, "records": count}
        if self.rank == 0:
            def u(x):
                return x & ((1 << 64) - 1)
            cross = 0
            prev = None
            for m, e in edges:
                if not m:
                    continue
                first, last = (u(e[0]), u(e[1])), (u(e[2]), u(e[3]))
                if prev is not None and first < prev:
                    cross += 1
                prev = last
            res["rank_boundary_violations"] = cross
            res["checksum_ok"] = (sum(cs) & ((1 << 64) - 1)) == checksum_in
            res["ok"] = tot_bad == 0 and cross == 0 and res["checksum_ok"] and count == self.total
        return res

    def checksum_global(self, rec: torch.Tensor) -> int:
        cs = D.gather_objects(TS.checksum(rec), 0, self.group)
        return (sum(cs) & ((1 << 64) - 1)) if self.rank == 0 else 0
