"""SPMD checkpoint/resume after a rank failure, CPU/gloo,
world size 2: the first launch runs an iterative word count whose rank 1 dies
(``MR_SPMD_FAULT=3:1:exit``) at the start of iteration 3 — the peers' collectives
fail, as after a lost GPU — and the relaunch (what ``torchrun --max-restarts``
does) resumes after iteration 2 from the manifest, finishes iterations 3 and 4
and produces the naive word counts.  A finished task starts again from scratch
(server.lua:469-502)."""
import json
import os
import socket

import torch.multiprocessing as mp

M = "lua_mapreduce_1_amd.examples.IterativeWordCount"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus():
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    return europarl_like(seed=5, lines=4_000, words=60_000, vocab_size=3_000, split_lines=500)


def _worker(rank, world, port, ckpt, state, fault, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_SPMD_FAULT=fault)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec

    _, _, device = D.init_from_env(backend="gloo", use_gpu=False, timeout_s=60)
    splits = _corpus()
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, checkpoint_dir=ckpt,
                          init_args={"nsplits": len(splits), "num_reducers": 5, "state_file": state,
                                     "iterations": 4}),
                     split_store=SplitStore(splits, pin=False), device=device)
    res = eng.run()
    gathered = eng.gather_results(res)
    if rank == 0:
        got = {}
        for _n, cols in gathered:
            for k, v in codec.iter_columnar(cols):
                got[k] = got.get(k, 0) + v[0]
        q.put((eng.resumed_from, eng.iteration, got))
    dist.barrier()
    dist.destroy_process_group()


def _launch(world, ckpt, state, fault, kill_after=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ckpt, state, fault, q)) for r in range(world)]
    for p in procs:
        p.start()
    if kill_after is not None:  # the failed rank exits; its peer errors out or is torn down
        procs[kill_after].join(240)
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.terminate()
                p.join(10)
        return [p.exitcode for p in procs], None
    for p in procs:
        p.join(240)
    return [p.exitcode for p in procs], q.get(timeout=5)


def test_spmd_resume_after_rank_failure(tmp_path):
    ckpt, state = str(tmp_path / "ckpt"), str(tmp_path / "state.json")
    codes, _ = _launch(2, ckpt, state, "3:1:exit", kill_after=1)
    assert codes[1] == 17 and codes[0] != 0, codes
    with open(os.path.join(ckpt, "result.spmd.json")) as f:
        m = json.load(f)
    assert m["iteration"] == 2 and not m["finished"]
    with open(state) as f:
        assert len(json.load(f)["totals"]) == 2

    codes, (resumed, iters, got) = _launch(2, ckpt, state, "")
    assert codes == [0, 0], codes
    assert resumed == 2 and iters == 4
    naive = {}
    for s in _corpus():
        for w in s.split():
            naive[w.decode()] = naive.get(w.decode(), 0) + 1
    assert got == naive
    with open(state) as f:
        totals = json.load(f)["totals"]
    assert totals == [sum(naive.values())] * 4
    with open(os.path.join(ckpt, "result.spmd.json")) as f:
        assert json.load(f)["finished"]

    # a finished task is not resumed: a new launch starts at iteration 1
    os.remove(state)
    codes, (resumed, iters, _got) = _launch(2, ckpt, state, "")
    assert codes == [0, 0] and resumed == 0 and iters == 4


def test_host_spmd_resume_in_process(tmp_path, monkeypatch):
    """The host-plane engine (reference-style mapfn) shares the manifest logic:
    a fault raised at the start of iteration 2 leaves iteration 1 recorded and
    a new engine resumes after it."""
    import sys
    mod = tmp_path / "hostiter.py"
    mod.write_text(
        "import json, os\n"
        "STATE = None\n"
        "def init(a):\n"
        "    global STATE\n"
        "    STATE = a['state']\n"
        "def taskfn(emit):\n"
        "    for i in range(1, 4):\n"
        "        emit(i, i)\n"
        "def mapfn(k, v, emit):\n"
        "    emit('sum', v)\n"
        "def partitionfn(k):\n"
        "    return 0\n"
        "def reducefn(k, vs, emit):\n"
        "    emit(sum(vs))\n"
        "def finalfn(pairs):\n"
        "    st = json.load(open(STATE)) if os.path.exists(STATE) else []\n"
        "    st += [v[0] for _k, v in pairs]\n"
        "    json.dump(st, open(STATE, 'w'))\n"
        "    return 'loop' if len(st) < 3 else True\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    from lua_mapreduce_1_amd import spmd
    from lua_mapreduce_1_amd.parallel.spmd_host import HostSPMDEngine
    state = str(tmp_path / "st.json")
    params = dict(taskfn="hostiter", mapfn="hostiter", partitionfn="hostiter", reducefn="hostiter",
                  finalfn="hostiter", init_args={"state": state}, checkpoint_dir=str(tmp_path / "ck"))
    monkeypatch.setenv("MR_SPMD_FAULT", "2:0:raise")
    eng = spmd(params)
    assert isinstance(eng, HostSPMDEngine)
    try:
        eng.run()
        raise AssertionError("fault not injected")
    except RuntimeError as e:
        assert "injected fault" in str(e)
    monkeypatch.delenv("MR_SPMD_FAULT")
    eng = spmd(params)
    eng.run()
    assert eng.resumed_from == 1 and eng.iteration == 3
    with open(state) as f:
        assert json.load(f) == [6, 6, 6]
    sys.modules.pop("hostiter", None)


def test_host_spmd_failed_job_after_retries(tmp_path, monkeypatch, capsys):
    """A map job that always raises is retried MAX_JOB_RETRIES times, then
    counted FAILED and left out of the results (server.lua:194-213)."""
    mod = tmp_path / "hostfail.py"
    mod.write_text(
        "CALLS = {}\n"
        "def taskfn(emit):\n"
        "    for i in range(1, 5):\n"
        "        emit(i, i)\n"
        "def mapfn(k, v, emit):\n"
        "    CALLS[k] = CALLS.get(k, 0) + 1\n"
        "    if k == 2:\n"
        "        raise ValueError('bad split')\n"
        "    emit('sum', v)\n"
        "def partitionfn(k):\n"
        "    return 0\n"
        "def reducefn(k, vs, emit):\n"
        "    emit(sum(vs))\n"
        "OUT = []\n"
        "def finalfn(pairs):\n"
        "    OUT.extend(pairs)\n"
        "    return True\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    monkeypatch.delenv("MR_SPMD_FAULT", raising=False)
    import importlib
    from lua_mapreduce_1_amd import spmd, utils
    eng = spmd(dict(taskfn="hostfail", mapfn="hostfail", partitionfn="hostfail", reducefn="hostfail",
                    finalfn="hostfail"), verbose=True)
    res = eng.run()
    m = importlib.import_module("hostfail")
    assert m.CALLS[2] == utils.MAX_JOB_RETRIES and m.CALLS[1] == 1
    assert res.failed_maps == 1 and m.OUT == [("sum", [1 + 3 + 4])]
    err = capsys.readouterr().err
    assert "# Failed maps     1" in err and "bad split" in err


def test_host_spmd_failed_reduce_after_retries(tmp_path, monkeypatch, capsys):
    """A reducefn that always raises for one partition: that reduce job is
    retried MAX_JOB_RETRIES times, counted FAILED and its partition dropped;
    the other partitions are reported (server.lua:194-213)."""
    mod = tmp_path / "hostredfail.py"
    mod.write_text(
        "CALLS = {}\n"
        "def taskfn(emit):\n"
        "    for i in range(1, 5):\n"
        "        emit(i, i)\n"
        "def mapfn(k, v, emit):\n"
        "    emit('k%d' % (v % 2), v)\n"
        "def partitionfn(k):\n"
        "    return int(k[1:])\n"
        "def reducefn(k, vs, emit):\n"
        "    CALLS[k] = CALLS.get(k, 0) + 1\n"
        "    if k == 'k1':\n"
        "        raise ValueError('bad reduce')\n"
        "    emit(sum(vs))\n"
        "OUT = []\n"
        "def finalfn(pairs):\n"
        "    OUT.extend(pairs)\n"
        "    return True\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    monkeypatch.delenv("MR_SPMD_FAULT", raising=False)
    import importlib
    from lua_mapreduce_1_amd import spmd, utils
    eng = spmd(dict(taskfn="hostredfail", mapfn="hostredfail", partitionfn="hostredfail", reducefn="hostredfail",
                    finalfn="hostredfail"), verbose=True)
    res = eng.run()
    m = importlib.import_module("hostredfail")
    assert m.CALLS["k1"] == utils.MAX_JOB_RETRIES and m.CALLS["k0"] == 1
    assert res.failed_reduces == 1 and m.OUT == [("k0", [2 + 4])]
    err = capsys.readouterr().err
    assert "# Failed reduces  1" in err and "bad reduce" in err


def test_manifest_key_covers_init_args_and_partitions():
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine
    e = SPMDEngine.__new__(SPMDEngine)
    e.world = 2
    e.params = dict(taskfn="t", mapfn="m", partitionfn="p", reducefn="r", finalfn="f", init_args={"a": 1})
    k1 = e._manifest_key()
    e.params = dict(e.params, init_args={"a": 2})
    k2 = e._manifest_key()
    e.params = dict(e.params, init_args={"a": 1}, num_partitions=7)
    k3 = e._manifest_key()
    assert k1 != k2 and k1 != k3 and k2 != k3


def _worker_restore(rank, world, port, ckpt, state, fault, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_SPMD_FAULT=fault)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec

    _, _, device = D.init_from_env(backend="gloo", use_gpu=False, timeout_s=30)
    splits = _corpus()
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, checkpoint_dir=ckpt,
                          init_args={"nsplits": len(splits), "num_reducers": 5, "state_file": state,
                                     "iterations": 4}),
                     split_store=SplitStore(splits, pin=False), device=device)
    res = eng.run()
    gathered = eng.gather_results(res)
    got = {}
    for _n, cols in gathered:
        for k, v in codec.iter_columnar(cols):
            got[k] = got.get(k, 0) + v[0]
    q.put((rank, eng.resumed_from, eng.iteration, eng.maps_restored, got if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def _launch_restore(world, ckpt, state, fault, expect_fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_restore, args=(r, world, port, ckpt, state, fault, q)) for r in range(world)]
    for p in procs:
        p.start()
    if expect_fail:
        procs[1].join(240)
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.terminate()
                p.join(10)
        return [p.exitcode for p in procs], None
    for p in procs:
        p.join(240)
    out = sorted((q.get(timeout=5) for _ in range(world)), key=lambda x: x[0])
    return [p.exitcode for p in procs], out


def test_spmd_restart_reruns_only_missing_maps(tmp_path):
    """Split-level restart: rank 1 dies at the start of
    iteration 3, after rank 0 finished and checkpointed its map of it; the
    relaunch resumes at iteration 3, rank 0 restores its map output instead of
    re-mapping its splits, rank 1 maps its own, and the counts are exact.
    Then a death after the map phase (``...:shuffle``): both ranks restore."""
    naive = {}
    for s in _corpus():
        for w in s.split():
            naive[w.decode()] = naive.get(w.decode(), 0) + 1
    for fault, restored in (("3:1:exit::start", [1, 0]), ("3:1:exit::shuffle", [1, 1])):
        d = tmp_path / fault.replace(":", "_")
        ckpt, state = str(d / "ckpt"), str(d / "state.json")
        codes, _ = _launch_restore(2, ckpt, state, fault, expect_fail=True)
        assert codes[1] == 17 and codes[0] != 0, codes
        maps = sorted(f for f in os.listdir(ckpt) if ".map.it3." in f)
        assert len(maps) == sum(restored), maps
        codes, out = _launch_restore(2, ckpt, state, "", expect_fail=False)
        assert codes == [0, 0], codes
        assert [o[1] for o in out] == [2, 2] and [o[2] for o in out] == [4, 4]
        assert [o[3] for o in out] == restored
        assert out[0][4] == naive
        with open(state) as f:
            assert json.load(f)["totals"] == [sum(naive.values())] * 4
        assert not [f for f in os.listdir(ckpt) if ".map." in f]  # consumed checkpoints are removed


def test_restored_map_keeps_failed_jobs(tmp_path):
    """a map checkpoint records the jobs that ended FAILED /
    BROKEN, so a restore reports the same failed maps (a failed job stays
    FAILED, /root/reference/mapreduce/server.lua:194-205)."""
    from lua_mapreduce_1_amd.parallel.spmd import JobRecord, SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils import STATUS
    splits = _corpus()
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, checkpoint_dir=str(tmp_path),
                          init_args={"nsplits": len(splits), "num_reducers": 5, "state_file": str(tmp_path / "s"),
                                     "iterations": 1}),
                     split_store=SplitStore(splits, pin=False), device="cpu")
    eng.iteration = 1
    recs = [JobRecord(i, None) for i in range(6)]
    for r in recs:
        r.status = STATUS.WRITTEN
    recs[2].status, recs[2].repetitions = STATUS.FAILED, 3
    recs[4].status, recs[4].repetitions = STATUS.BROKEN, 1
    eng._save_job_status(recs, 0, 6)
    back = [JobRecord(i, None) for i in range(6)]
    eng._restore_job_status(back, 0, 6)
    assert [r.status for r in back] == [STATUS.WRITTEN, STATUS.WRITTEN, STATUS.FAILED, STATUS.WRITTEN,
                                        STATUS.BROKEN, STATUS.WRITTEN]
    assert back[2].repetitions == 3
    eng._drop_map_ckpt(1)
    assert not os.listdir(tmp_path) or all(".jobs." not in f for f in os.listdir(tmp_path))
