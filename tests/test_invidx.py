"""Inverted index as a MapReduce job (examples/InvertedIndex; BASELINE config
"inverted-index build on the same corpus shape"): word -> sorted distinct line
numbers through the framework's own roles — the SPMD engine's list plane
(parallel/planes.py) on CPU (1 rank), over gloo (3 ranks), on the GPU (HIP
kernels; 1 rank, several ranks sharing it, the forced RCCL shuffle) and the
server/worker roles (host mapfn/reducefn) — each diffed against a naive
oracle."""
import contextlib
import io
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

M = "lua_mapreduce_1_amd.examples.InvertedIndex"


def _splits(seed=9):
    from lua_mapreduce_1_amd.utils.corpus import europarl_like, tricky_text
    s = europarl_like(seed=seed, lines=3000, words=60000, vocab_size=3000, split_lines=500)
    s.append(tricky_text(np.random.default_rng(seed), 150_000))
    s.append(b"no trailing newline here")
    s.append(b"ends with space ")
    s.append(b"word word word\nword\n\n\nlast")
    return s


def _engine(splits, device, nred=7, **extra):
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"nsplits": len(splits), "num_reducers": nred}, **extra)
    return spmd(params, device=device, split_store=SplitStore(splits, pin=torch.device(device).type == "cuda"))


def _result():
    import importlib
    return importlib.import_module(M).RESULT


def _naive(splits):
    import importlib
    return importlib.import_module(M).naive_index(splits)


def test_cpu_single_rank_matches_oracle():
    splits = _splits()
    eng = _engine(splits, "cpu")
    res = eng.run()
    exp = _naive(splits)
    assert _result() == exp
    assert res.total_value == sum(len(v) for v in exp.values())
    # result files named like every job's, keys in order inside each
    for name, cols in eng.gather_results(res):
        assert name.startswith("result.P")
        from lua_mapreduce_1_amd.runtime import codec
        keys = [k.encode("utf-8", "surrogateescape") for k, _ in codec.iter_columnar(cols)]
        assert keys == sorted(keys)


@pytest.mark.parametrize("windowed", [False, True])
def test_split_files_number_lines_like_the_oracle(tmp_path, windowed):
    """SplitStore.from_files (execute_spmd --split-glob) pads a
    file with a newline only when it does not end in a newline, like the
    in-memory store and the oracle — a file ending in '\n' gains no empty
    line, so later line ids do not shift; one ending in a space does (ADVICE
    r3: its last line and the next file's first line are different lines)."""
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore, WindowedSplitStore
    splits = _splits()
    paths = []
    for i, b in enumerate(splits):
        p = tmp_path / f"s{i:03d}.txt"
        p.write_bytes(b)
        paths.append(str(p))
    store = SplitStore.from_files(paths, pin=False)
    assert len(store) == len(splits)
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"nsplits": len(splits), "num_reducers": 5})
    if windowed:
        # the windowed store (inputs larger than host memory) has the same layout
        ws = WindowedSplitStore(paths, window_mb=64)
        assert ws.offsets.tolist() == store.offsets.tolist()
    spmd(params, device="cpu", split_store=store).run()
    assert _result() == _naive(splits)


def test_trailing_space_file_ends_its_line(tmp_path):
    """A split ending in a space is followed by a newline: the next split's
    first line is a new global line."""
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd import SplitStore
    splits = [b"alpha beta ", b"gamma\ndelta ", b"eps"]
    assert _naive(splits) == {"alpha": [0], "beta": [0], "gamma": [1], "delta": [2], "eps": [3]}
    paths = []
    for i, b in enumerate(splits):
        p = tmp_path / f"t{i}.txt"
        p.write_bytes(b)
        paths.append(str(p))
    for store in (SplitStore(splits, pin=False), SplitStore.from_files(paths, pin=False)):
        params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                      init_args={"nsplits": len(splits), "num_reducers": 3})
        spmd(params, device="cpu", split_store=store).run()
        assert _result() == _naive(splits)


def test_server_worker_host_plane_matches_oracle(tmp_path):
    """The same module through server + worker (host mapfn reads its split
    file, reducefn = sorted distinct lines) — the reference deployment."""
    import lua_mapreduce_1_amd as mr
    from lua_mapreduce_1_amd.runtime import coordinator
    splits = _splits()
    files = []
    for i, s in enumerate(splits):
        p = tmp_path / f"s{i:03d}.txt"
        p.write_bytes(s)
        files.append(str(p))
    cs = coordinator.start_local()
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, combinerfn=M, storage="gridfs",
                  device="auto", init_args={"files": files, "num_reducers": 5})
    s = mr.server.new(cs, "invidx_sw")
    s.poll_sleep = 0.02
    s.quiet = True
    s.configure(params)
    w = mr.worker.new(cs, "invidx_sw")
    w.configure(verbose=False, poll_sleep=0.02, max_iter=2)
    t = threading.Thread(target=w.execute, daemon=True)
    t.start()
    with contextlib.redirect_stdout(io.StringIO()):
        s.loop()
    assert _result() == _naive(splits)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, on_gpu=False, backend="gloo", force_shuffle=False, pipelined=False):
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
    splits = _splits()
    extra = {"table_capacity": 1 << 16}
    if force_shuffle:
        extra["force_shuffle"] = True
    eng = _engine(splits, device, **extra)
    if pipelined:
        # three iterations with prefetched inputs and each next map queued
        # early (own stream, vocabulary and sink), every result checked
        from lua_mapreduce_1_amd.runtime import codec
        eng.prefetch, eng.pipeline = True, True
        want, same = _naive(splits), True
        for i in range(3):
            res = eng.run_iteration(prefetch_next=i < 2, lookahead=2 - i)
            parts = eng.gather_results(res)
            if rank == 0:
                same &= {k: v for _n, c in parts for k, v in codec.iter_columnar(c)} == want
        own_ok = all(p % world == rank for p in res.result_names) and eng.plane._states[1] is not None
        oks = D.gather_objects(own_ok, 0)
        if rank == 0:
            q.put((same, all(oks)))
        dist.barrier()
        dist.destroy_process_group()
        return
    res = eng.run()
    own_ok = all(p % world == rank for p in res.result_names)
    oks = D.gather_objects(own_ok, 0)
    if rank == 0:
        q.put((_result() == _naive(splits), all(oks)))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    same, owned = q.get(timeout=300)
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert same and owned


@pytest.mark.parametrize("world", [3])
def test_gloo_multi_rank_matches_oracle(world):
    _run(world)


def test_gloo_forced_shuffle_one_rank():
    _run(1, force_shuffle=True)


@pytest.mark.gpu
def test_gpu_single_rank_matches_oracle(gpu):
    splits = _splits()
    eng = _engine(splits, gpu, table_capacity=1 << 16)
    res = eng.run()
    assert res.device["docs"].is_cuda
    assert _result() == _naive(splits)
    # a second iteration on the same engine (tables reset, staging reused)
    eng.finished = False
    res = eng.run_iteration()
    got = {k: v for _n, c in eng.gather_results(res) for k, v in __import__(
        "lua_mapreduce_1_amd.runtime.codec", fromlist=["x"]).iter_columnar(c)}
    assert got == _naive(splits)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [False, True])
def test_gpu_staged_chunks_and_prefetch(gpu, pipeline):
    """Small copy chunks mapped as their copies land (line numbers continue
    across chunks), and iterations whose copies were prefetched during the
    previous iteration's sort — with ``pipeline`` also each next iteration's
    map queued (own stream, vocabulary and sink) while this one is ordered."""
    from lua_mapreduce_1_amd.runtime import codec
    splits = _splits()
    eng = _engine(splits, gpu, table_capacity=1 << 16)
    eng.chunk_bytes = [8 << 10, 16 << 10, 32 << 10]
    eng.tail_bytes = [8 << 10]
    eng.prefetch, eng.pipeline = True, pipeline
    want = _naive(splits)
    for i in range(4):
        res = eng.run_iteration(prefetch_next=i < 3, lookahead=3 - i)
        got = {k: v for _n, c in eng.gather_results(res) for k, v in codec.iter_columnar(c)}
        assert got == want
    assert not eng._inflight
    assert (eng.plane._states is not None and eng.plane._states[1] is not None) == pipeline


@pytest.mark.gpu
def test_gpu_long_lines_and_many_lines(gpu):
    """Lines longer than a tile / chunk, and more lines than one tile's worth."""
    rng = np.random.default_rng(4)
    words = [b"w%d" % i for i in range(500)]
    long_line = b" ".join(words[i % 500] for i in rng.integers(0, 500, 30000)) + b"\n"
    many = b"".join(b"%s %s\n" % (words[i % 500], words[(i * 7) % 500]) for i in range(40000))
    splits = [long_line, many, long_line[:70000] + b"\n" + many[:50000]]
    _engine(splits, gpu, table_capacity=1 << 14).run()
    assert _result() == _naive(splits)


@pytest.mark.gpu
def test_gpu_dense_one_letter_tokens(gpu):
    """Tiles with more tokens than the map kernel buffers (one-letter words:
    up to 4096 tokens per 8 KiB tile > 2048) take the direct-write path."""
    rng = np.random.default_rng(5)
    letters = [bytes([c]) for c in b"abcdefghijklmnopqrstuvwxyz0123456789"]
    lines = [b" ".join(letters[i] for i in rng.integers(0, len(letters), int(n))) + b"\n"
             for n in rng.integers(1, 3000, 120)]
    splits = [b"".join(lines[:60]), b"".join(lines[60:])]
    _engine(splits, gpu, table_capacity=1 << 12).run()
    assert _result() == _naive(splits)


@pytest.mark.gpu
def test_gpu_multi_rank_on_one_gpu(gpu):
    _run(2, on_gpu=True)


@pytest.mark.gpu
def test_gpu_multi_rank_pipelined(gpu):
    """Two ranks sharing the GPU (gloo) running pipelined list-plane iterations."""
    _run(2, on_gpu=True, pipelined=True)


@pytest.mark.gpu
def test_gpu_forced_shuffle_rccl(gpu):
    """The list plane's three all_to_all_single on the RCCL backend (one-rank
    nccl group, W>1 path forced)."""
    _run(1, on_gpu=True, backend="nccl", force_shuffle=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 300_000, 1_500_000])
def test_gpu_sort_unique_matches_torch(gpu, n):
    """keys-only radix sort + fused two-pass unique == torch.unique (sorted)."""
    from lua_mapreduce_1_amd.ops import invidx as II
    from lua_mapreduce_1_amd.ops.primitives import sort_keys
    g = torch.Generator().manual_seed(n)
    keys = torch.randint(0, max(2, n // 3), (n,), generator=g, dtype=torch.int64) << 7
    keys |= torch.randint(0, 3, (n,), generator=g, dtype=torch.int64)
    got = II.sort_unique(keys.to(gpu), 40).cpu()
    assert torch.equal(got, torch.unique(keys))
    _, sk = sort_keys([keys.to(gpu)], bits=[40], return_keys=True, keys_only=True)
    assert torch.equal(sk.cpu(), torch.sort(keys).values)


@pytest.mark.gpu
def test_gpu_seg_gather_matches_cpu(gpu):
    from lua_mapreduce_1_amd.ops import invidx as II
    g = torch.Generator().manual_seed(3)
    lens = torch.randint(0, 50, (2000,), generator=g)
    lens[7] = 100_000  # one very frequent word
    starts = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens, 0)])
    docs = torch.randint(0, 1 << 30, (int(starts[-1]),), generator=g, dtype=torch.int32)
    perm = torch.randperm(2000, generator=g)
    nl = lens[perm]
    noff = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(nl, 0)])
    want = II.seg_gather(perm, starts, noff, docs)
    got = II.seg_gather(perm.to(gpu), starts.to(gpu), noff.to(gpu), docs.to(gpu)).cpu()
    assert torch.equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("unique", [True, False])
@pytest.mark.parametrize("n", [1, 4095, 4096, 300_001])
def test_group_words_matches_split_words(gpu, unique, n):
    """The fused count/scatter word grouping (ops/invidx.group_words) equals
    unique (concat_unique) + split_words on sorted posting keys with repeated
    postings, tile-crossing words and a doc base."""
    from lua_mapreduce_1_amd.ops import invidx as II
    g = torch.Generator().manual_seed(n)
    doc_bits, id_bits = 12, 10
    words = torch.randint(0, 1 << id_bits, (n,), generator=g)
    docs = torch.randint(0, 1 << 9, (n,), generator=g)  # small: many repeats
    keys = torch.sort((words << doc_bits) | docs).values
    ref_keys = torch.unique(keys) if unique else keys
    rw, rs, rd = II.split_words(ref_keys, doc_bits, id_bits, 7)
    gw, gs, gd = II.group_words(keys.to(gpu), doc_bits, id_bits, 7, unique=unique)
    assert torch.equal(gw.cpu(), rw) and torch.equal(gs.cpu(), rs) and torch.equal(gd.cpu(), rd)


def _restart_rank(rank, world, port, q, ckpt, fault):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_SPMD_FAULT=fault)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    D.init_from_env(backend="gloo", use_gpu=False, timeout_s=30)
    splits = _splits()
    eng = _engine(splits, torch.device("cpu"), checkpoint_dir=ckpt)
    eng.run()
    if rank == 0:
        q.put((rank, eng.maps_restored, _result() == _naive(splits)))
    else:
        q.put((rank, eng.maps_restored, None))
    dist.barrier()
    dist.destroy_process_group()


def test_list_restart_restores_postings(tmp_path):
    """Split-level restart on the list plane: rank 1 dies after the map phase
    (``1:1:exit::shuffle``); both ranks had saved their postings, and the
    relaunch restores them instead of re-mapping, with the oracle's index."""
    ckpt = str(tmp_path / "ckpt")
    ctx = mp.get_context("spawn")

    def launch(fault, fail):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_restart_rank, args=(r, 2, port, q, ckpt, fault)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            if p.is_alive():
                p.terminate()
                p.join(10)
        return [p.exitcode for p in procs], (None if fail else sorted(q.get(timeout=5) for _ in range(2)))

    codes, _ = launch("1:1:exit::shuffle", True)
    assert codes[1] == 17 and codes[0] != 0, codes
    assert len([f for f in os.listdir(ckpt) if ".map.it1." in f]) == 2
    codes, out = launch("", False)
    assert codes == [0, 0], codes
    assert [o[1] for o in out] == [1, 1] and out[0][2] is True


def _restart_gpu_proc(q, ckpt, fault):
    os.environ["MR_SPMD_FAULT"] = fault
    splits = _splits()
    eng = _engine(splits, torch.device("cuda", 0), table_capacity=1 << 16, checkpoint_dir=ckpt)
    eng.run()
    q.put((eng.maps_restored, _result() == _naive(splits)))


@pytest.mark.gpu
def test_list_restart_restores_postings_gpu(gpu, tmp_path):
    ckpt = str(tmp_path / "ckpt")
    ctx = mp.get_context("spawn")
    for fault, want_code in (("1:0:exit::shuffle", 17), ("", 0)):
        q = ctx.Queue()
        p = ctx.Process(target=_restart_gpu_proc, args=(q, ckpt, fault))
        p.start()
        p.join(180)
        assert p.exitcode == want_code, p.exitcode
    restored, ok = q.get(timeout=5)
    assert restored == 1 and ok


def _device_order_ok(res, R):
    """res.device (the list plane's device result) holds every partition's
    words in exact bytewise order, long words sharing a prefix included."""
    out = res.device
    koff = out["key_off"].cpu().numpy()
    blob = out["key_blob"].cpu().numpy().tobytes()
    counts = out["counts_host"]
    a = 0
    for c in counts:
        keys = [blob[koff[i]:koff[i + 1]] for i in range(a, a + c)]
        if keys != sorted(keys):
            return False
        a += c
    return a == len(koff) - 1


def _long_prefix_splits():
    import numpy as np
    rng = np.random.default_rng(5)
    words = [b"sharedprefix_" + bytes(rng.integers(97, 123, size=int(rng.integers(1, 12))).astype(np.uint8))
             for _ in range(400)] + [b"sharedprefix_", b"short", b"a"]
    lines = [b" ".join(words[int(i)] for i in rng.integers(0, len(words), size=12)) for _ in range(3000)]
    return [b"\n".join(lines[i:i + 500]) + b"\n" for i in range(0, 3000, 500)]


@pytest.mark.parametrize("on_gpu", [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_device_result_in_exact_key_order(request, on_gpu):
    dev = request.getfixturevalue("gpu") if on_gpu else "cpu"
    splits = _long_prefix_splits()
    eng = _engine(splits, dev, nred=3, **({"table_capacity": 1 << 16} if on_gpu else {}))
    res = eng.run_iteration()
    assert _device_order_ok(res, 3)
    from lua_mapreduce_1_amd.runtime import codec
    got = {k: v for _n, c in eng.gather_results(res) for k, v in codec.iter_columnar(c)}
    assert got == _naive(splits)
