#!/usr/bin/env python
"""Shuffle time of the SPMD host plane (plain ``mapfn`` modules,
parallel/spmd_host.py) at W gloo ranks on the CPU: the tests' host word count
(tests/host_modules.py: string and tuple keys) over a larger corpus.  Every
rank maps its jobs once; then, after a barrier, the same map output is
shuffled by the engine's one-collective byte all-to-all (_shuffle_host) and
by the round-4 shuffle (W scatter_object_list rounds of pickled dicts,
``legacy`` below), alternately; prints the slowest rank's times.

    python tools/host_shuffle_w8.py [--world 8] [--lines 80000] [--iters 5]
"""
import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _rank(rank, world, port, q, lines, iters):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_NUMA_BIND="0")
    import torch
    torch.set_num_threads(1)
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel import dist as D
    _, _, device = D.init_from_env(backend="gloo", use_gpu=False)
    import torch.distributed as tdist
    from lua_mapreduce_1_amd.parallel.spmd import assign_contiguous
    from lua_mapreduce_1_amd.runtime import modules
    M = "host_modules"
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, init_args={"lines": lines}), device=device)
    jobs = eng._jobs()
    j0, j1 = assign_contiguous([1] * len(jobs), rank, world)
    local: dict = {}
    part = modules.field(eng.partmod, "partitionfn")
    for j in range(j0, j1):
        for p, kv in eng._map_job(jobs[j][0], jobs[j][1], None, part).items():
            dst = local.setdefault(p, {})
            for k, v in kv.items():
                dst.setdefault(k, []).extend(v)

    def legacy(local, failed):
        send = [dict() for _ in range(world)]
        for p, kv in local.items():
            send[p % world][p] = kv
        recv = [None] * world
        for src in range(world):
            out = [None]
            tdist.scatter_object_list(out, send if rank == src else None, src=src)
            recv[src] = out[0]
        mine: dict = {}
        for piece in recv:
            for p, kv in piece.items():
                dst = mine.setdefault(p, {})
                for k, v in kv.items():
                    dst.setdefault(k, []).extend(v)
        return mine, D.all_reduce_sum_int(failed, device)

    times = {"new": [], "legacy": []}
    ref = None
    for _ in range(iters):
        for name, fn in (("new", eng._shuffle_host), ("legacy", legacy)):
            D.barrier()
            t0 = time.perf_counter()
            mine, _f = fn(local, 0)
            times[name].append(D.all_reduce_max(time.perf_counter() - t0, device))
            got = {p: {k: sorted(v, key=repr) for k, v in kv.items()} for p, kv in mine.items()}
            assert ref is None or got == ref
            ref = got
    if rank == 0:
        q.put((times, sum(len(kv) for kv in local.values())))
    D.barrier()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--lines", type=int, default=80_000)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t0 = time.time()
    ps = [ctx.Process(target=_rank, args=(r, a.world, port, q, a.lines, a.iters)) for r in range(a.world)]
    for p in ps:
        p.start()
    times, nkeys = q.get(timeout=600)
    for p in ps:
        p.join(60)
    for name, sh in times.items():
        sh_ms = [round(1e3 * x, 1) for x in sh]
        print(f"world {a.world}, {a.lines} lines, {nkeys} keys on rank 0: {name:6s} shuffle ms (slowest rank) "
              f"{sh_ms}, median {sorted(sh_ms)[len(sh_ms) // 2]}")
    print(f"(wall {time.time() - t0:.1f} s)")


if __name__ == "__main__":
    main()
