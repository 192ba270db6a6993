"""TeraSort as a MapReduce job (examples/TeraSort; BASELINE config
"TeraSort-style 10 GB key/value sort"): TeraGen map jobs, sampled range
partitioner, all-to-all of 100-byte rows and the identity reduce's radix sort
through the SPMD engine's record plane — checked for global order and an
order-independent record checksum on CPU, over gloo (2 and 4 ranks, forced
shuffle), on the GPU (HIP kernels vs the NumPy specification, forced RCCL
shuffle) and through server/worker."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lua_mapreduce_1_amd.ops import terasort as TS


def test_generator_layout_and_keys():
    r = TS.generate(50, 1000, 99)
    a = r.numpy()
    assert a.shape == (50, 100)
    assert int.from_bytes(bytes(a[3, 10:18]), "little") == 1003
    hi, lo = TS.keys(r)
    assert int(hi[0]) & ((1 << 64) - 1) == int.from_bytes(bytes(a[0, :8]), "big")
    assert int(lo[0]) == int.from_bytes(bytes(a[0, 8:10]), "big")
    # same records regardless of how the range is split
    assert torch.equal(TS.generate(20, 1010, 99), r[10:30])


M = "lua_mapreduce_1_amd.examples.TeraSort"


def _engine(records, device, blocks=3, partitions=0, **extra):
    from lua_mapreduce_1_amd import spmd
    return spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                     init_args={"records": records, "blocks": blocks, "partitions": partitions, "validate": True},
                     **extra), device=device)


def _validation():
    import importlib
    return importlib.import_module(M).VALIDATION


@pytest.mark.parametrize("partitions", [1, 4])
def test_cpu_single_rank_sort(partitions):
    """TeraGen map jobs -> sampled range partitions -> identity reduce; the
    gathered result files are globally sorted in file-name order."""
    from lua_mapreduce_1_amd.runtime import codec
    eng = _engine(30000, "cpu", partitions=partitions)
    res = eng.run()
    assert _validation()["ok"], _validation()
    keys = [k.encode("utf-8", "surrogateescape") for _n, c in eng.gather_results(res)
            for k, _v in codec.iter_columnar(c)]
    assert len(keys) == 30000 and keys == sorted(keys)
    assert len(res.result_names) == partitions


def test_record_store_input_and_server_worker_host_plane():
    """A caller-staged RecordStore input; and the same module through the
    server/worker roles (host TeraGen map, uniform static splitters)."""
    import contextlib
    import io
    import threading
    import lua_mapreduce_1_amd as mr
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.planes import RecordStore
    from lua_mapreduce_1_amd.runtime import coordinator
    blocks = [TS.generate(4000, 0, 0x7E5A), TS.generate(3000, 4000, 0x7E5A)]
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                    init_args={"records": 7000, "blocks": 2, "partitions": 3, "validate": True}),
               device="cpu", split_store=RecordStore(blocks))
    eng.run()
    assert _validation()["ok"]
    cs = coordinator.start_local()
    s = mr.server.new(cs, "terasort_sw")
    s.poll_sleep = 0.02
    s.quiet = True
    s.configure(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, storage="gridfs", device="auto",
                     init_args={"records": 3000, "blocks": 3, "partitions": 2}))
    w = mr.worker.new(cs, "terasort_sw")
    w.configure(verbose=False, poll_sleep=0.02, max_iter=2)
    threading.Thread(target=w.execute, daemon=True).start()
    with contextlib.redirect_stdout(io.StringIO()):
        s.loop()
    assert _validation() == {"records": 3000, "ok": True}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, on_gpu=False, backend="gloo", force_shuffle=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import datetime
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    if force_shuffle:
        dist.init_process_group(backend, rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120),
                                **({"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}))
        device = torch.device("cuda", 0) if on_gpu else torch.device("cpu")
    else:
        _, _, device = D.init_from_env(backend=backend, use_gpu=on_gpu)
    extra = {"oversample": 256}
    if force_shuffle:
        extra["force_shuffle"] = True
    eng = _engine(40001, device, blocks=max(world, 2), **extra)
    eng.run()
    if rank == 0:
        q.put(_validation())
    dist.barrier()
    dist.destroy_process_group()


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    v = q.get(timeout=300)
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert v["ok"], v


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_multi_rank_sort(world):
    _run(world)


def test_gloo_forced_shuffle_one_rank():
    _run(1, force_shuffle=True)


@pytest.mark.gpu
def test_gpu_kernels_match_numpy(gpu):
    rc = TS.generate(5000, 77, 1234)
    rg = TS.generate(5000, 77, 1234, gpu)
    assert torch.equal(rg.cpu(), rc)
    hc, lc = TS.keys(rc)
    hg, lg = TS.keys(rg)
    assert torch.equal(hg.cpu(), hc) and torch.equal(lg.cpu(), lc)
    assert TS.checksum(rg) == TS.checksum(rc)
    sp = torch.tensor([-(1 << 62), 0, 1 << 62], dtype=torch.int64)
    assert torch.equal(TS.dest_of(hg, sp).cpu(), TS.dest_of(hc, sp))
    perm = torch.randperm(5000, dtype=torch.int32)
    assert torch.equal(TS.gather(rg, perm.to(gpu)).cpu(), rc[perm.long()])


@pytest.mark.gpu
def test_gpu_keys_digit_histograms_feed_the_sort(gpu):
    """Key extraction with histograms: digits 4..7 of hi equal numpy's counts
    (digits 0..3 untouched), and the sort fed with them gives the same
    permutation as the sort that computes its own."""
    n = 3_000_017
    rg = TS.generate(n, 5, 99, gpu)
    gh = torch.zeros(2048, dtype=torch.int32, device=gpu)
    hg, lg = TS.keys(rg, gh)
    top = (hg.cpu().numpy().view(np.uint64) >> np.uint64(32)).astype(np.uint64)
    want = np.zeros((8, 256), np.int64)
    for b in range(4):
        want[4 + b] = np.bincount(((top >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.int64), minlength=256)
    assert np.array_equal(gh.cpu().numpy().reshape(8, 256), want)
    assert torch.equal(TS.sort_perm(hg, lg, gh), TS.sort_perm(hg, lg))


@pytest.mark.gpu
@pytest.mark.parametrize("partitions", [1, 3])
def test_gpu_single_rank_sort(gpu, partitions):
    eng = _engine(300_007, gpu, blocks=2, partitions=partitions)
    res = eng.run()
    assert _validation()["ok"], _validation()
    out = res.device["records"]
    assert out.is_cuda
    k = out[:2000, :10].cpu().numpy()
    assert [bytes(x) for x in k] == sorted(bytes(x) for x in k)


@pytest.mark.gpu
def test_gpu_multi_rank_on_one_gpu(gpu):
    _run(2, on_gpu=True)


@pytest.mark.gpu
def test_gpu_forced_shuffle_rccl(gpu):
    """The record plane's all_to_all_single of 100-byte rows on RCCL."""
    _run(1, on_gpu=True, backend="nccl", force_shuffle=True)


@pytest.mark.gpu
@pytest.mark.parametrize("mod", [200_000, 50, 0])
def test_gpu_sort_perm_with_prefix_ties(gpu, mod):
    """Equal 8-byte prefixes: short runs go through the tie fix-up kernel,
    long runs (mod=50) through the full (hi, lo) fallback; both stable."""
    g = torch.Generator().manual_seed(mod + 1)
    n = 300_000
    hi = torch.randint(-2**63, 2**63 - 1, (n,), generator=g, dtype=torch.int64)
    if mod:
        hi = hi % mod
    lo = torch.randint(0, 1 << 16, (n,), generator=g, dtype=torch.int64)
    ref = TS.sort_perm(hi, lo)
    got = TS.sort_perm(hi.to(gpu), lo.to(gpu)).cpu().long()
    assert torch.equal(got, ref.long())


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uniform", "runs", "skewed"])
def test_gpu_sort_perm_top32_fixup(gpu, case):
    """sort_perm sorts only the top 32 bits of hi and fixes runs of equal top
    bits by (hi, lo): uniform keys, many short runs (2..40 rows sharing the
    top 32 bits), and a skewed key set whose runs exceed the fix-up limit
    (full-sort fallback) all give the exact 80-bit order."""
    g = np.random.default_rng({"uniform": 1, "runs": 2, "skewed": 3}[case])
    n = 200_000
    hi = g.integers(0, 2**63, n, dtype=np.int64).view(np.uint64) * np.uint64(2) + g.integers(0, 2, n).astype(np.uint64)
    if case == "runs":
        top = g.integers(0, n // 20, n).astype(np.uint64) << np.uint64(32)
        hi = top | (hi & np.uint64(0xFFFFFFFF))
    elif case == "skewed":
        hi = (np.uint64(7) << np.uint64(32)) | (hi & np.uint64(0xFFFF))
    lo = g.integers(0, 1 << 16, n).astype(np.uint64)
    th = torch.from_numpy(hi.view(np.int64)).to(gpu)
    tl = torch.from_numpy(lo.view(np.int64)).to(gpu)
    perm = TS.sort_perm(th, tl).cpu().numpy().astype(np.int64)
    want = np.lexsort((lo, hi))
    assert np.array_equal(hi[perm], hi[want]) and np.array_equal(lo[perm], lo[want])
