#!/usr/bin/env python
"""Per-rank proxy of TeraSort at W ranks on ONE GPU (BASELINE.json config
"TeraSort-style 10 GB key/value sort on 8xMI355X"): rank 0 of a simulated
world of W ranks holds 1/W of the 10 GB (100-byte records generated in HBM)
and runs the record plane's whole W>1 path — key pass, splitter sampling,
partition, exchange, receive-side sort and gather.  The collectives are a
model: what peer p sends rank 0 is computed before timing from peer p's own
TeraGen block (its rows of rank 0's range, in the order the exchange being
measured sends them: distinct keys, the real receive-side work), copied in
on a copy stream beside an exchange stream that holds for bytes /
``--xgmi-gbs`` (the all-to-all's link time; the exchange ends when both are
done, and the next one starts after it), so an asynchronous exchange overlaps
the compute stream as RCCL's would.

Both W>1 exchanges of the record plane, selected by MR_REC_CHUNKS: K >= 1
(round 6) = the exchange pipelined by key range (K rounds, each round's
received rows sorted on their own while later rounds are on the wire); 0
(round 5) = stable sort by destination, one exchange, one key sort of
everything received.

    python tools/proxy_terasort.py --world 8 [--gb 10] [--steps 10] [--xgmi-gbs 400]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lua_mapreduce_1_amd import spmd  # noqa: E402
from lua_mapreduce_1_amd.ops import records as RC  # noqa: E402
from lua_mapreduce_1_amd.ops import terasort as TS  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402
from lua_mapreduce_1_amd.parallel import planes as PL  # noqa: E402
from lua_mapreduce_1_amd.parallel import spmd as S  # noqa: E402
from lua_mapreduce_1_amd.parallel.planes import RecordStore  # noqa: E402
from lua_mapreduce_1_amd.utils.config import TUNABLES  # noqa: E402

M = "lua_mapreduce_1_amd.examples.TeraSort"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--gb", type=float, default=10.0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--xgmi-gbs", type=float, default=400.0,
                    help="modelled all-to-all bytes/s leaving (and entering) one GPU, GB/s")
    a = ap.parse_args()
    W = a.world
    device = torch.device("cuda", 0)
    total = int(a.gb * 1e9) // 100
    mod = importlib.import_module(M)
    mod.init({"records": total, "blocks": W})
    blocks = mod.blocks()
    first, n0 = blocks[0]
    store = RecordStore([TS.generate(n0, first, mod.SEED, device)] +
                        [torch.empty((n, TS.REC), dtype=torch.uint8, device="meta") for _f, n in blocks[1:]])

    # -- the exchange model ---------------------------------------------------
    xs = torch.cuda.Stream(device)
    # torch.cuda._sleep spins for a number of shader clocks: calibrate to ms
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(10_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles_per_ms = 10_000_000 / e0.elapsed_time(e1)
    peers = []  # [peer][round] -> the rows peer p sends rank 0 in that round, filled before timing
    K = min(max(0, int(TUNABLES.rec_chunks)), 1024 // W)

    def link_hold(nbytes: int) -> None:
        ms = nbytes / (a.xgmi_gbs * 1e9) * 1e3
        if ms > 0:
            torch.cuda._sleep(int(ms * cycles_per_ms))

    peer_counts = []  # device [W-1][rounds]: filled with peers

    def exchange_counts(counts, group=None):
        c = counts.view(W, -1).clone()  # [source][rounds..., failed maps]
        if peer_counts:
            c[1:, :-1] = peer_counts[0]
        else:  # (the run that finds the splitters: peers send what rank 0 sends itself)
            c[1:, :-1] = c[0, :-1]
        c[1:, -1] = c[0, -1]
        return c.reshape(-1)

    cats = []  # [round] -> peers 1..W-1's rows of that round, concatenated (filled with peers)
    cats_k32 = []  # [round] -> their 32-bit key prefixes (shipped beside the rows on the GPU)

    def fill(out, payload, own, k):
        """out <- [this rank's own rows (or key prefixes) of round k | peer 1's | ...] (two copies)"""
        out[:own].copy_(payload[:own])
        src = cats if payload.dim() == 2 else cats_k32
        if src:
            m = min(src[k].shape[0], out.shape[0] - own)
            out[own:own + m].copy_(src[k][:m])

    xc = torch.cuda.Stream(device)  # the model's copy of the transfer's bytes (beside the link hold)

    def exchange(out, payload, send, k):
        """One all-to-all on the model's streams: the copy (xc) and the link
        hold (xs) run side by side — the transfer takes the longer of the two
        — and after the previous exchange (one all-to-all at a time, as on
        RCCL's stream).  Returns its completion event."""
        cur = torch.cuda.current_stream()
        xs.wait_stream(cur)
        xc.wait_stream(cur)
        xc.wait_stream(xs)
        with torch.cuda.stream(xc):
            fill(out, payload, send[0], k)
            evc = torch.cuda.Event()
            evc.record(xc)
        with torch.cuda.stream(xs):
            link_hold((sum(send) - send[0]) * payload[:1].numel() * payload.element_size())
            xs.wait_event(evc)
            ev = torch.cuda.Event()
            ev.record(xs)
        payload.record_stream(xc)
        out.record_stream(xc)
        return ev

    def all_to_all_v(payload, send, recv, group=None):
        out = torch.empty((sum(recv),) + tuple(payload.shape[1:]), dtype=payload.dtype, device=payload.device)
        torch.cuda.current_stream().wait_event(exchange(out, payload, send, 0))
        return out

    class _Work:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    rnd = [0, 0]  # rounds of row exchanges, of key-prefix exchanges

    def all_to_all_v_into(out, payload, send, recv, group=None, async_op=False):
        j = 0 if payload.dim() == 2 else 1
        k = rnd[j] % max(K, 1)
        rnd[j] += 1
        return _Work(exchange(out, payload, send, k))

    def all_gather_tensor(t, group=None):
        return t.repeat((W,) + (1,) * (t.dim() - 1))

    D.exchange_counts = exchange_counts
    D.all_to_all_v = all_to_all_v
    D.all_to_all_v_into = all_to_all_v_into
    D.all_gather_tensor = all_gather_tensor
    S.D.world_info = lambda group=None: (0, W)
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"records": total, "blocks": W, "partitions": W})
    eng = spmd(params, device=device, split_store=store)
    assert eng.world == W and eng.rank == 0
    # the splitters of rank 0's sample, then every peer's rows of rank 0's
    # range from its own block, per round, in the order the exchange sends them
    res = eng.run_iteration()
    sp, sub = res.device["splitters"], res.device.get("subsplitters")
    del res
    for p in range(1, W):
        fp, npp = blocks[p]
        blk = TS.generate(npp, fp, mod.SEED, device)
        k32 = RC.keys32(blk, TS.KEY)
        if K >= 1:
            s = RC.dest32(k32, sub).to(torch.int64)
            peers.append([blk[s == k] for k in range(K)])
        else:
            peers.append([blk[RC.dest32(k32, sp).to(torch.int64) == 0]])
        del blk, k32
    cats.extend(torch.cat([pr[k] for pr in peers]) for k in range(len(peers[0])))
    cats_k32.extend(RC.keys32(c, TS.KEY) for c in cats)
    peer_counts.append(torch.tensor([[r.shape[0] for r in pr] for pr in peers], dtype=torch.int64, device=device))
    for _ in range(a.warmup):
        rnd[0] = rnd[1] = 0
        res = eng.run_iteration()
        del res
    torch.cuda.synchronize()
    per = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t1 = time.perf_counter()
        rnd[0] = rnd[1] = 0
        res = eng.run_iteration()
        torch.cuda.synchronize()
        per.append(1000 * (time.perf_counter() - t1))
        timings = res.timings
        out = res.device["records"]
        del res
    ms = 1000 * (time.perf_counter() - t0) / a.steps
    # the rank's output must be in key order and hold every row of its range
    ok = RC.unsorted_pairs(out, TS.KEY) == 0
    own = RC.keys32(TS.generate(n0, first, mod.SEED, device), TS.KEY)
    mine = int((RC.dest32(own, sp).to(torch.int64) == 0).sum())
    rows_ok = int(out.shape[0]) == mine + sum(r.shape[0] for pr in peers for r in pr)
    per.sort()
    print(json.dumps({"proxy": "terasort per-rank", "world": W, "gb_total": a.gb, "rows_in": n0,
                      "rows_out": int(out.shape[0]), "rows_ok": rows_ok,
                      "rounds": K, "xgmi_gbs_model": a.xgmi_gbs, "ms_per_step": ms, "median": per[len(per) // 2],
                      "min": per[0], "sorted": ok,
                      "phases_ms": {k: round(1000 * v, 3) for k, v in timings.items()}}), flush=True)
    return 0 if ok and rows_ok else 3


if __name__ == "__main__":
    sys.exit(main())
