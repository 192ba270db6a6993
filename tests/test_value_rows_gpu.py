"""GPU variants of tests/test_value_rows.py: tuple and byte-string values on
the general device plane (HIP list-mode insert of k-word value rows, value
bytes gathered and shuffled through RCCL), against the host oracles."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_generic_plane import _free_port, run_engine  # noqa: E402
from test_value_rows import PI, SI, _pi_got, pi_data, si_data  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lua_mapreduce_1_amd.ops import _hip
    _hip.lib()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("which", ["pi", "si"])
def test_value_rows_gpu_w1(gpu, which):
    import importlib
    mod = PI if which == "pi" else SI
    splits = pi_data() if which == "pi" else si_data()
    eng, res, got = run_engine(mod, splits, gpu, {"num_reducers": 7})
    assert eng.device.type == "cuda" and eng.plane.map.table.is_cuda
    exp = importlib.import_module(mod).naive(splits)
    assert (_pi_got(got) if which == "pi" else got) == exp


def _rank(port, q, which):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import datetime
    import importlib
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            timeout=datetime.timedelta(seconds=120), device_id=dev)
    mod = PI if which == "pi" else SI
    splits = pi_data() if which == "pi" else si_data()
    eng, res, got = run_engine(mod, splits, dev, {"num_reducers": 7}, force_shuffle=True)
    exp = importlib.import_module(mod).naive(splits)
    q.put(((_pi_got(got) if which == "pi" else got) == exp, res.bytes_shuffled))
    dist.destroy_process_group()


@pytest.mark.parametrize("which", ["pi", "si"])
def test_value_rows_rccl_forced_shuffle(gpu, which):
    """The W>1 path on one GPU (one-rank nccl group): value rows and value
    bytes through RCCL all_to_all_single."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank, args=(_free_port(), q, which))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    ok, shipped = q.get(timeout=5)
    assert ok and shipped > 0


def test_device_reducefn_over_bytes_gpu(gpu, monkeypatch):
    """device_reducefn over ByteValues on the GPU: per word the number of
    distinct sources, counted by hashing the value bytes on the device."""
    import importlib
    from lua_mapreduce_1_amd.ops import segments as S
    from lua_mapreduce_1_amd.parallel.values import ByteValues
    m = importlib.import_module(SI)

    def device_reducefn(keys, off, val):
        assert isinstance(val, ByteValues) and val.blob.is_cuda
        return S.count(off)
    monkeypatch.setattr(m, "device_reducefn", device_reducefn, raising=False)
    monkeypatch.setattr(m, "device_reduce", None)
    def combinerfn(key, values, emit):  # host combiner over str values (NOT the reducer: device_reducefn
        m.reducefn(key, values, emit)    # is not its batched form), then the device reducer
    monkeypatch.setattr(m, "combinerfn", combinerfn)
    splits = si_data()
    eng, res, got = run_engine(SI, splits, gpu, {"num_reducers": 5})
    exp = m.naive(splits)
    assert got == {k: [len(v)] for k, v in exp.items()}
