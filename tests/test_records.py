"""The record plane for rows of any width (record widths as
parameters): 64-byte rows with 16-byte keys, 37-byte rows (not a multiple of
4) with 5-byte keys, TeraSort's 100/10, and skewed keys (the full-key
fallback of the 32-bit prefix sort) — W = 1, forced shuffle and gloo W = 3 on
CPU; the GPU kernels against the CPU specification in test_records_gpu."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
M = "rec_modules"
SHAPES = [dict(rb=64, kb=16), dict(rb=37, kb=5), dict(rb=100, kb=10), dict(rb=24, kb=3, skew=True)]
IDS = ["64x16", "37x5", "100x10", "24x3-skew"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def expected(args):
    import importlib
    mod = importlib.import_module(M)
    mod.init(dict(args, rows=args.get("rows", 10000)))
    rows = np.concatenate([mod.block_rows(b) for b in range(mod.BLOCKS)])
    return rows, mod.KB


def check(got_rows: np.ndarray, args) -> bool:
    rows, kb = expected(args)
    if got_rows.shape != rows.shape:
        return False
    keys = [bytes(r[:kb]) for r in got_rows]
    if keys != sorted(keys):
        return False
    a = np.sort(rows.view(np.dtype((np.void, rows.shape[1]))).ravel())
    b = np.sort(got_rows.view(np.dtype((np.void, rows.shape[1]))).ravel())
    return bool(np.array_equal(a, b))


def run_engine(args, device, **params):
    from lua_mapreduce_1_amd import spmd
    eng = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, init_args=dict(args), **params), device=device)
    res = eng.run_iteration()
    parts = eng.gather_results(res)
    rows = np.concatenate([c["records"] for _n, c in parts]) if parts else None
    return eng, res, rows


@pytest.mark.parametrize("args", SHAPES, ids=IDS)
def test_records_any_width_cpu(args):
    eng, res, rows = run_engine(args, torch.device("cpu"))
    assert eng.plane_kind == "records" and check(rows, args)
    assert len(res.result_names) == (4 if not args.get("skew") else len(res.result_names))


def test_records_shape_must_agree():
    from lua_mapreduce_1_amd.parallel.planes import RecordEmitter

    class P:
        shape = None
        _out: list = []
        _take = staticmethod(lambda rec: None)

        class eng:
            device = torch.device("cpu")
    e = RecordEmitter(P)
    e.records(torch.zeros((3, 8), dtype=torch.uint8), 4)
    with pytest.raises(ValueError):
        e.records(torch.zeros((3, 9), dtype=torch.uint8), 4)
    with pytest.raises(ValueError):
        RecordEmitter(type("Q", (), {"shape": None, "_out": [], "_take": staticmethod(lambda r: None),
                                     "eng": P.eng})).records(
            torch.zeros((3, 8), dtype=torch.uint8), 9)


def _rank(rank, world, port, q, args, force_shuffle, extra=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import datetime
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    if force_shuffle:
        dist.init_process_group("gloo", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                                timeout=datetime.timedelta(seconds=120))
    else:
        D.init_from_env(backend="gloo", use_gpu=False)
    eng, _res, rows = run_engine(args, torch.device("cpu"), force_shuffle=force_shuffle, **(extra or {}))
    if rank == 0:
        q.put(check(rows, args) and (not extra or eng.plane._spilled))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,force", [(3, False), (1, True)], ids=["gloo3", "forced1"])
@pytest.mark.parametrize("args", [SHAPES[1], SHAPES[3]], ids=["37x5", "24x3-skew"])
def test_records_multi_rank_cpu(args, world, force):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, args, force)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5)


# -- spill tier: rows beyond the HBM cap -------------------------
SPILL = [dict(rb=64, kb=16, rows=20000), dict(rb=37, kb=5, rows=20000), dict(rb=24, kb=3, skew=True, rows=20000)]
SPILL_IDS = ["64x16", "37x5", "24x3-skew"]


@pytest.mark.parametrize("args", SPILL, ids=SPILL_IDS)
def test_records_spill_external_sort_cpu(args):
    """1.3 MB of rows under a 0.1 MB cap: spilled to host, bucket pass,
    per-bucket sorts; the output equals a sort of the input."""
    eng, res, rows = run_engine(args, torch.device("cpu"), record_cap_mb=0.1)
    assert eng.plane._spilled and res.device["spilled"]
    assert check(rows, args)


@pytest.mark.parametrize("world,force", [(3, False), (1, True)], ids=["gloo3", "forced1"])
def test_records_spill_multi_rank_cpu(world, force):
    args = SPILL[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, args, force, {"record_cap_mb": 0.05}))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5)


def test_host_rounds_cover_every_row():
    from lua_mapreduce_1_amd.parallel.planes import _host_rounds
    blocks = [torch.arange(n * 7, dtype=torch.int64).to(torch.uint8).view(n, 7) for n in (5, 0, 13, 1, 40)]
    rounds = _host_rounds(blocks, 50)
    assert all(sum(p.numel() for p in r) <= 50 for r in rounds)
    assert torch.equal(torch.cat([p for r in rounds for p in r]), torch.cat(blocks))


@pytest.mark.gpu
@pytest.mark.parametrize("args", SPILL, ids=SPILL_IDS)
def test_records_spill_external_sort_gpu(gpu, args):
    a = dict(args, rows=200_000)
    eng, res, rows = run_engine(a, gpu, record_cap_mb=1.0)
    assert eng.plane._spilled and res.device["spilled"]
    assert check(rows, a)


# -- GPU kernels vs the CPU specification ---------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("args", SHAPES, ids=IDS)
def test_records_any_width_gpu(gpu, args):
    from lua_mapreduce_1_amd.ops import records as RC
    rows, kb = expected(dict(args, rows=300_000))
    h = torch.from_numpy(rows)
    d = h.to(gpu)
    assert torch.equal(RC.keys32(d, kb).cpu(), RC.keys32(h, kb))
    hh, hl = RC.keys(h, kb)
    dh, dl = RC.keys(d, kb)
    assert torch.equal(dh.cpu(), hh) and torch.equal(dl.cpu(), hl)
    perm, _ = RC.sort(d, kb)
    out = RC.gather(d, perm).cpu().numpy()
    assert check(out, dict(args, rows=300_000))
    ref = torch.from_numpy(np.lexsort((hl.numpy().view(np.uint64), hh.numpy().view(np.uint64))))
    assert torch.equal(RC.gather(d, ref.to(gpu)).cpu(), h[ref])  # the gather itself
    eng, res, got = run_engine(dict(args, rows=200_000), gpu)
    assert check(got, dict(args, rows=200_000))


@pytest.mark.gpu
@pytest.mark.parametrize("rb", [4, 12, 16, 20, 24, 36, 37, 64, 100, 116, 128, 132, 244, 248])
def test_record_gather_widths_gpu(gpu, rb):
    """records.gather (16-byte LDS-staged path for 16 <= rb <= 244, rb % 4 == 0;
    dword / byte gathers otherwise and with mode=1) against torch indexing:
    row counts that are not a multiple of the 256-row batch, repeated and
    reversed rows, a permutation longer than the input."""
    from lua_mapreduce_1_amd.ops import records as RC
    g = torch.Generator().manual_seed(rb)
    nin = 70_001
    rec = torch.randint(0, 256, (nin, rb), dtype=torch.uint8, generator=g)
    d = rec.to(gpu)
    perms = [torch.randperm(nin, generator=g), torch.arange(nin - 1, -1, -1),
             torch.randint(0, nin, (nin + 517,), generator=g), torch.randint(0, nin, (255,), generator=g)]
    for p in perms:
        want = rec[p]
        for mode in (0, 1):
            got = RC.gather(d, p.to(torch.int32).to(gpu), mode=mode).cpu()
            assert torch.equal(got, want), (rb, mode, p.numel())
    # a view whose base is not 16-byte aligned takes the dword path
    if rb % 4 == 0 and nin > 2:
        flat = d.view(-1)[4:4 + (nin - 1) * rb].view(nin - 1, rb)
        p = torch.randperm(nin - 1, generator=g)
        assert torch.equal(RC.gather(flat, p.to(gpu)).cpu(), rec.view(-1)[4:4 + (nin - 1) * rb].view(nin - 1, rb)[p])


def _restart_rank(rank, world, port, q, args, ckpt, fault):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_SPMD_FAULT=fault)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    D.init_from_env(backend="gloo", use_gpu=False, timeout_s=30)
    eng, _res, rows = run_engine(args, torch.device("cpu"), checkpoint_dir=ckpt)
    q.put((rank, eng.maps_restored, check(rows, args) if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_records_restart_restores_rows(tmp_path):
    """Split-level restart on the record plane: rank 1 dies after the map
    phase (``1:1:exit::shuffle``); both ranks had saved their rows, and the
    relaunch restores them instead of re-running the map jobs."""
    ckpt = str(tmp_path / "ckpt")
    args = dict(SHAPES[0], rows=20_000)
    ctx = mp.get_context("spawn")

    def launch(fault, fail):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_restart_rank, args=(r, 2, port, q, args, ckpt, fault)) for r in range(2)]
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


def _restart_gpu_proc(q, args, ckpt, fault):
    os.environ["MR_SPMD_FAULT"] = fault
    eng, _res, rows = run_engine(args, torch.device("cuda", 0), checkpoint_dir=ckpt)
    q.put((eng.maps_restored, check(rows, args)))


@pytest.mark.gpu
def test_records_restart_restores_rows_gpu(gpu, tmp_path):
    ckpt = str(tmp_path / "ckpt")
    args = dict(SHAPES[2], rows=50_000)
    ctx = mp.get_context("spawn")
    for fault, want_code in (("1:0:exit::shuffle", 17), ("", 0)):
        q = ctx.Queue()
        p = ctx.Process(target=_restart_gpu_proc, args=(q, args, ckpt, fault))
        p.start()
        p.join(180)
        assert p.exitcode == want_code, p.exitcode
    restored, ok = q.get(timeout=5)
    assert restored == 1 and ok


@pytest.mark.gpu
@pytest.mark.parametrize("rb", [100, 64, 24, 244, 8])
def test_row_gathers_equal_gpu(gpu, rb):
    """The 16-byte LDS-staged row gather and the dword gather move the same
    bytes as a host gather of a full row permutation."""
    from lua_mapreduce_1_amd.ops import records as RC
    n = 100_003
    g = torch.Generator().manual_seed(rb)
    rec = torch.randint(0, 256, (n, rb), dtype=torch.uint8, generator=g).to(gpu)
    perm = torch.randperm(n, generator=g).to(torch.int32).to(gpu)
    assert torch.equal(RC.gather(rec, perm, mode=1), RC.gather(rec, perm, mode=0))
    assert torch.equal(RC.gather(rec, perm, mode=0).cpu(), rec.cpu()[perm.cpu().long()])


@pytest.mark.parametrize("fmt", ["legacy", "unknown"])
def test_records_checkpoint_formats(tmp_path, fmt):
    """a map checkpoint of the round-3 format (one ``rows`` array +
    ``key_bytes``) is restored; a file of an unknown format is ignored and the
    map re-runs — a relaunch never dies on KeyError('shape')."""
    ckpt = str(tmp_path / "ckpt")
    args = dict(SHAPES[0], rows=6000)
    eng, _res, rows = run_engine(args, torch.device("cpu"), checkpoint_dir=ckpt)
    assert check(rows, args)
    # iteration 2 of a new engine on the same checkpoint dir: plant its map checkpoint
    from lua_mapreduce_1_amd import spmd
    eng2 = spmd(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, init_args=dict(args), checkpoint_dir=ckpt),
                device=torch.device("cpu"))
    eng2.iteration = 0
    eng2.iteration += 1
    path = eng2._map_ckpt_path()
    eng2.iteration -= 1
    want, kb = expected(args)
    with open(path, "wb") as f:
        if fmt == "legacy":
            np.savez(f, rows=want, key_bytes=np.array([kb], np.int64))
        else:
            np.savez(f, something=np.zeros(3))
    res = eng2.run_iteration()
    got = np.concatenate([c["records"] for _n, c in eng2.gather_results(res)])
    assert check(got, args)
    assert eng2.maps_restored == (1 if fmt == "legacy" else 0)


