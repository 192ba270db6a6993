"""The SPMD statistics block at W > 1 covers every rank's jobs (the
reference aggregates over all job documents, server.lua:155-183,538-600):
``Map sum(real_time)`` is the sum of each rank's own map jobs, the cluster
and server times are the slowest rank's, distinct keys are summed over the
ranks' disjoint partitions (gloo, W = 3, fold and general planes)."""
import os
import re
import socket

import pytest
import torch
import torch.multiprocessing as mp

WC = "lua_mapreduce_1_amd.models.wordcount"
SS = "lua_mapreduce_1_amd.examples.ScoreStats"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, mod):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils.corpus import europarl_like, score_csv
    D.init_from_env(backend="gloo", use_gpu=False)
    if mod == SS:
        splits = score_csv(seed=3, lines=9000, vocab_size=800, split_lines=1000)
    else:
        splits = europarl_like(seed=9, lines=9000, words=120_000, vocab_size=5000, split_lines=1000)
    eng = SPMDEngine(dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod,
                          init_args={"nsplits": len(splits), "num_reducers": 7}),
                     split_store=SplitStore(splits, pin=False), device=torch.device("cpu"))
    res = eng.run_iteration()
    block = eng.stats_block(res)
    mine = [r for r in res.map_jobs if r.worker == rank]
    q.put((rank, sum(r.real_time for r in mine), sum(r.cpu_time for r in mine), res.timings["iteration"],
           res.distinct_keys, len(mine), block))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mod", [WC, SS], ids=["fold", "general"])
def test_stats_block_sums_every_rank(mod):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, mod)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted((q.get(timeout=5) for _ in range(world)), key=lambda x: x[0])
    assert sum(g[5] for g in got) == 9  # every split mapped by exactly one rank
    blocks = [g[6] for g in got]
    assert len(set(blocks)) == 1  # every rank prints the same global block

    def val(key):
        m = re.search(re.escape(key) + r"\s+([0-9.eE+-]+)", blocks[0])
        return float(m.group(1))
    assert val("Map sum(real_time)") == pytest.approx(sum(g[1] for g in got), abs=2e-6)
    assert val("Map sum(cpu_time)") == pytest.approx(sum(g[2] for g in got), abs=2e-6)
    assert val("Server time") == pytest.approx(max(g[3] for g in got), abs=2e-6)
    assert val("Distinct keys") == sum(g[4] for g in got)
    assert "# Ranks 3" in blocks[0]
