"""The driver's bench.py contract on CPU: world size 1 and 2 (torchrun, gloo,
127.0.0.1 rendezvous) on a reduced corpus — exactly one JSON line from rank 0
with the required keys, whole-job words/s, and every token counted."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(cmd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_bench_json_contract_cpu(n):
    args = ["bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1", "--lines", "4000", "--words", "60000"]
    if n == 1:
        out = _run([sys.executable] + args)
    else:
        out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                    "--master-addr", "127.0.0.1", "--master-port", "29611"] + args)
    assert KEYS <= set(out)
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["valid"] is True and out["config"]["words"] == 60000
    assert out["value"] > 0 and out["higher_is_better"] is True
    assert "REDUCED" in out["data"]
    assert out["world"] == n and out["backend"] in ("gloo", "single-process-cpu")
    assert out["config"]["per_key_valid"] is True
    assert out["cold_first_iteration_ms"] > 0


def test_bench_spawns_its_own_ranks_cpu():
    """``python bench.py --gpus 2`` with no torchrun environment starts the two
    ranks itself and relays rank 0's single JSON line (the driver's N>1 form
    must never silently measure one rank)."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--lines", "4000",
                "--words", "60000"])
    assert out["n_gpus"] == 2 and out["world"] == 2 and out["backend"] == "gloo"
    assert out["config"]["valid"] is True and out["config"]["per_key_valid"] is True
