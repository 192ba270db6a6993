"""The DP-SGD example (examples/DigitsMLP, the reference's APRIL-ANN job:
/root/reference/mapreduce/examples/APRIL-ANN/common.lua:85-202) through the
SPMD MapReduce engine's tensor plane (parallel/tensor_plane.py; VERDICT r4
#4): per-weight fp32 gradients emitted as tensors, summed by a reduce-scatter
by weight-name partition + an all-gather, the optimizer step in
``device_finalfn`` on every rank.  Its loss history must match the direct
trainer ``models/mlp_dpsgd.train_spmd`` within fp32 tolerance: CPU at W = 1
and gloo W = 4 (here), GPU at W = 1 and through a one-rank RCCL group
(test_digits_spmd_gpu below, marked gpu)."""
import math
import os
import socket
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DM = "lua_mapreduce_1_amd.examples.DigitsMLP"
REF_PNG = "/root/reference/misc/digits.png"
EPOCHS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data_arg():
    return REF_PNG if os.path.exists(REF_PNG) else "synthetic"


def run_digits(device, data, epochs=EPOCHS, force_shuffle=False):
    import importlib
    from lua_mapreduce_1_amd import spmd
    m = importlib.import_module(DM)
    eng = spmd(dict(taskfn=DM, mapfn=DM, partitionfn=DM, reducefn=DM, finalfn=DM,
                    init_args={"data": data, "max_epochs": epochs}, force_shuffle=force_shuffle), device=device)
    assert eng.plane_kind == "tensor"
    res = eng.run()
    return list(m.HISTORY), eng, res


def reference_history(device, data, epochs=EPOCHS, graphs=False):
    from lua_mapreduce_1_amd.models import mlp_dpsgd as T
    from lua_mapreduce_1_amd.utils import digits
    out = T.train_spmd(device, data=digits.load(None if data == "synthetic" else data), epochs=epochs, graphs=graphs)
    return out["history"]


def close(h1, h2, rel=2e-4) -> bool:
    if len(h1) != len(h2):
        return False
    for a, b in zip(h1, h2):
        for k in ("tr_loss", "va_loss"):
            if not math.isclose(a[k], b[k], rel_tol=rel, abs_tol=1e-6):
                return False
        if abs(a["va_acc"] - b["va_acc"]) > 0.011 or a["epoch"] != b["epoch"]:
            return False
    return True


def test_digits_tensor_plane_cpu_w1():
    data = _data_arg()
    hist, eng, res = run_digits(torch.device("cpu"), data)
    ref = reference_history("cpu", data)
    assert close(hist, ref), (hist, ref)
    assert res.failed_maps == 0 and len(res.result_names) == len({sum(k.encode()) % 10 for k in
                                                                  ("w1", "b1", "w2", "b2", "TR_LOSS")})


def _rank(rank, world, port, q, data):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MR_NUMA_BIND="0")
    torch.set_num_threads(1)
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    D.init_from_env(backend="gloo", use_gpu=False)
    hist, eng, res = run_digits(torch.device("cpu"), data)
    owned = sorted(res.result_names)
    allowned = D.gather_objects(owned, 0)
    if rank == 0:
        q.put((hist, allowned))
    dist.barrier()
    dist.destroy_process_group()


def test_digits_tensor_plane_gloo_w4():
    """Four ranks, one map job each: the same history as one process running
    the four bunches (the sums only change their fp32 order); each weight
    name reduced by the rank owning its partition."""
    import torch.multiprocessing as mp
    data = _data_arg()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 4, port, q, data)) for r in range(4)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    hist, allowned = q.get(timeout=5)
    assert close(hist, reference_history("cpu", data)), hist
    parts = sorted(p for o in allowned for p in o)
    assert parts == sorted({sum(k.encode()) % 10 for k in ("w1", "b1", "w2", "b2", "TR_LOSS")})
    assert all(p % 4 == r for r, o in enumerate(allowned) for p in o)


def test_digits_execute_spmd_cli(tmp_path):
    """The module through execute_spmd.py's positional interface (one
    process: world size 1)."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, MR_NUMA_BIND="0", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(root, "execute_spmd.py"), "--device", "cpu", DM, DM, DM, DM, DM,
                        "nil", "nil", json.dumps({"data": "synthetic", "max_epochs": 2})],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.gpu
def test_digits_tensor_plane_gpu():
    """GPU: the MFMA gradient kernel's per-job gradients through the tensor
    plane vs the direct trainer (eager and hipGraph-replayed)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    hist, eng, res = run_digits(dev, "synthetic", epochs=6)
    assert res.tensors["w1"].is_cuda
    assert close(hist, reference_history(dev, "synthetic", epochs=6, graphs=False))
    assert close(hist, reference_history(dev, "synthetic", epochs=6, graphs=True))


def _rccl_rank(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import datetime
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            timeout=datetime.timedelta(seconds=120), device_id=dev)
    hist, eng, res = run_digits(dev, "synthetic", epochs=4, force_shuffle=True)
    q.put(close(hist, reference_history(dev, "synthetic", epochs=4)))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_digits_tensor_plane_rccl_one_gpu():
    """The RCCL reduce-scatter + all-gather path on the box's one GPU (a
    one-rank nccl group with the shuffle forced)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    p.start()
    p.join(300)
    assert p.exitcode == 0 and q.get(timeout=5)
