"""Multi-rank SPMD engine on CPU (gloo), world sizes 2 and 3: the all-to-all
shuffle, partition ownership (p % W) and the gathered final results must match
a naive single-process word count."""
import os
import socket

import pytest
import torch.multiprocessing as mp

M = "lua_mapreduce_1_amd.models.wordcount"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, on_gpu=False, pipelined=False, backend="gloo", force_shuffle=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like

    if force_shuffle:
        # a one-rank group: init_from_env skips it at W = 1
        import datetime
        dist.init_process_group(backend, rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120),
                                **({"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}))
        device = torch.device("cuda", 0) if on_gpu else torch.device("cpu")
    else:
        _, _, device = D.init_from_env(backend=backend, use_gpu=on_gpu)
    splits = europarl_like(seed=9, lines=12_000, words=200_000, vocab_size=8_000, split_lines=1000)
    store = SplitStore(splits, pin=on_gpu)
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                          init_args={"nsplits": len(splits), "num_reducers": 7}, force_shuffle=force_shuffle),
                     split_store=store, device=device)
    if force_shuffle:
        assert dist.get_backend() == backend
    if on_gpu:
        assert eng.table.is_cuda
    if pipelined:  # iteration i+1's copies and map overlap iteration i's shuffle/reduce
        eng.prefetch = eng.pipeline = True
        for i in range(4):
            res = eng.run_iteration(prefetch_next=i < 3, lookahead=3 - i)
        assert eng._pending is None and not eng._inflight
    else:
        res = eng.run()
    owned = sorted(res.partitions)
    assert all(p % world == rank for p in owned)
    gathered = eng.gather_results(res)
    if rank == 0:
        got = {}
        for _name, cols in gathered:
            for k, v in codec.iter_columnar(cols):
                got[k] = got.get(k, 0) + v[0]
        naive = {}
        for s in splits:
            for w in s.split():
                k = w.decode()
                naive[k] = naive.get(k, 0) + 1
        names = [n for n, _ in gathered]
        q.put((got == naive, names == sorted(names), len(got)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_spmd_gloo_wordcount(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, sorted_names, n = q.get(timeout=5)
    assert ok and sorted_names and n > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("world,pipelined", [(2, False), (4, False), (3, True)])
def test_spmd_multirank_on_one_gpu(world, pipelined):
    """Several ranks share the GPU (gloo carries the collectives through host
    copies): exercises the device shuffle/reduce/finalize kernels at W > 1,
    also with pipelined iterations (next map on a second stream)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, True, pipelined)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, sorted_names, n = q.get(timeout=5)
    assert ok and sorted_names and n > 1000


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, sorted_names, n = q.get(timeout=5)
    assert ok and sorted_names and n > 1000


def test_spmd_forced_shuffle_one_rank_gloo():
    """MR_FORCE_SHUFFLE / force_shuffle: the W>1 data path (pack, count
    exchange, all-to-all, receive-side reduce) at world size 1."""
    _run(1, force_shuffle=True)


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [False, True])
def test_spmd_forced_shuffle_rccl_one_gpu(pipelined):
    """The RCCL branch of the shuffle (dist._a2a -> all_to_all_single on the
    nccl backend, device buffers) on the single GPU of the box: a one-rank
    nccl group with the W>1 path forced, checked against the naive count."""
    _run(1, on_gpu=True, backend="nccl", force_shuffle=True, pipelined=pipelined)


def _single_sync_worker(port, q, mode):
    """One-rank nccl group, W>1 path forced, pipelined iterations: host waits
    per iteration and every iteration's result against the naive count."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    if mode == "device_error":
        os.environ["MR_SPMD_DEVICE_FAULT"] = "3:1"  # the chunk of job 3 fails once (device error word)
    import datetime
    import torch
    import torch.distributed as dist
    from lua_mapreduce_1_amd.ops import _hip
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            timeout=datetime.timedelta(seconds=120), device_id=torch.device("cuda", 0))
    splits = europarl_like(seed=9, lines=12_000, words=200_000, vocab_size=8_000, split_lines=1000)
    naive = {}
    for s in splits:
        for w in s.split():
            naive[w.decode()] = naive.get(w.decode(), 0) + 1
    store = SplitStore(splits, pin=True)
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                          init_args={"nsplits": len(splits), "num_reducers": 7}, force_shuffle=True),
                     split_store=store, device=torch.device("cuda", 0),
                     table_capacity=1024 if mode == "map_overflow" else 1 << 20)
    eng.prefetch = eng.pipeline = True
    waits, ok = [], []
    n_it = 6
    for i in range(n_it):
        if i == 3 and mode == "send_bound":
            eng._send_est = 100      # the compaction's bound is too small: flagged, exchange redone
            eng._send_cap_test = 4096  # and its send buffer (the bound sizes it with room to spare)
        if i == 3 and mode == "red_bound":
            eng._red_distinct = 100  # the padded tail's bound is too small: TailBoundError, tail re-run
        w0 = _hip.WAITS[0]
        res = eng.run_iteration(prefetch_next=i < n_it - 1, lookahead=2)
        got = {}
        for _n, cols in eng.gather_results(res):
            for k, v in codec.iter_columnar(cols):
                got[k] = got.get(k, 0) + v[0]
        waits.append(_hip.WAITS[0] - w0)
        ok.append(got == naive)
    q.put((ok, waits, eng._single_sync_ok(True, True)))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["steady", "send_bound", "red_bound", "map_overflow", "device_error"])
def test_single_sync_iteration_rccl_one_gpu(mode):
    """a W>1 fold-plane iteration waits on the device twice
    (count exchange with the map's checks; result download), every result
    exact; the redo paths (send bound, reduce bound, map overflow, device
    error word) stay exact and only add waits to the iteration they hit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_single_sync_worker, args=(_free_port(), q, mode))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    ok, waits, single = q.get(timeout=5)
    assert single and all(ok), (ok, waits)
    steady = [w for i, w in enumerate(waits) if i >= 1 and not (mode != "steady" and i == 3)]
    if mode in ("map_overflow", "device_error"):
        steady = waits[4:]
    assert max(steady) <= 2, waits


def _long_keys_worker(port, q):
    """One-rank nccl group, W>1 path forced, keys that overlap in their
    source (tests/long_key_modules.py): the send buffer sized from the row
    bound is too small for their key bytes every iteration."""
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import datetime
    from collections import Counter
    import torch
    import torch.distributed as dist
    import long_key_modules as LK
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            timeout=datetime.timedelta(seconds=120), device_id=torch.device("cuda", 0))
    # long lines (60 words): nearly every window is WIDTH bytes long
    splits = europarl_like(seed=9, lines=2_000, words=120_000, vocab_size=8_000, split_lines=250)
    want = Counter(w.decode("utf-8", "surrogateescape") for s in splits for w in LK.windows(s))
    L = "long_key_modules"
    eng = SPMDEngine(dict(taskfn=L, mapfn=L, partitionfn=L, reducefn=L, finalfn=L,
                          init_args={"nsplits": len(splits), "num_reducers": 7}, force_shuffle=True),
                     split_store=SplitStore(splits, pin=True), device=torch.device("cuda", 0))
    # the first exchange sized from a small row bound (a fresh process: the
    # reused send buffer has not been grown by an earlier, larger bound)
    eng._send_est = 100
    ok = []
    for i in range(3):
        res = eng.run_iteration()
        got = {}
        for _n, cols in eng.gather_results(res):
            for k, v in codec.iter_columnar(cols):
                got[k] = got.get(k, 0) + v[0]
        ok.append(got == want)
    q.put((ok, eng._single_sync_ok(True, True), getattr(eng, "_send_cap_min", 0)))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_single_sync_send_capacity_redo_long_keys():
    """a capacity redo of the single-sync count exchange grows the
    send buffer from the exchanged per-destination totals, so keys whose bytes
    exceed the bound-derived capacity finish (they looped forever before)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_long_keys_worker, args=(_free_port(), q))
    p.start()
    p.join(240)
    if p.exitcode is None:
        p.kill()
    assert p.exitcode == 0
    ok, single, floor = q.get(timeout=5)
    assert single and all(ok) and floor > 0, (ok, single, floor)
