"""SPMD launcher: run a user MapReduce task with one process per GPU, the data
plane in HBM and the shuffle over RCCL (parallel/spmd.py) — the same user
modules and positional arguments as execute_server.lua, minus the connection
string and database (there is no job queue to share):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        [--max-restarts 3] -m lua_mapreduce_1_amd.cli.execute_spmd \\
        [--checkpoint-dir DIR] [--device auto|cpu] [--num-partitions R] [--split-glob G]... [-v] \\
        TASKFN MAPFN PARTITIONFN REDUCEFN [FINALFN|nil] [COMBINERFN|nil] [STORAGE|nil] [INIT_ARGS...]

One process (no torchrun) runs world size 1.  ``--checkpoint-dir`` makes an
iterative task resume after its last finished iteration when torchrun
relaunches the ranks after a failure (``--max-restarts``).  A map module
with a ``device_mapfn`` runs on the HIP data plane (parallel/spmd.py); a
plain ``mapfn`` runs the reference's host semantics on every rank
(parallel/spmd_host.py).  STORAGE is accepted for parity and ignored (the
shuffle goes over collectives).  INIT_ARGS are passed to every module's
``init`` (execute_server.lua:50); a single JSON object argument is decoded.
"""
from __future__ import annotations

import argparse
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="execute_spmd")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--device", default="auto", choices=("auto", "cpu"))
    ap.add_argument("--num-partitions", type=int, default=None)
    ap.add_argument("--result-ns", default=None)
    ap.add_argument("--split-glob", action="append", default=[],
                    help="split files (sorted, in order of the options) that map modules with "
                         "device_input='split' read; each rank loads only its own share; repeatable")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("taskfn")
    ap.add_argument("mapfn")
    ap.add_argument("partitionfn")
    ap.add_argument("reducefn")
    ap.add_argument("rest", nargs="*")
    a = ap.parse_args(argv)
    rest = list(a.rest)
    finalfn = rest.pop(0) if rest else None
    combinerfn = rest.pop(0) if rest else None
    _storage = rest.pop(0) if rest else None  # accepted for CLI parity: SPMD ranks shuffle over collectives
    finalfn = None if finalfn == "nil" else finalfn
    combinerfn = None if combinerfn == "nil" else combinerfn
    init_args = rest
    if len(rest) == 1 and rest[0].startswith("{"):
        init_args = json.loads(rest[0])
    try:
        sys.stdout.reconfigure(errors="surrogateescape")
    except AttributeError:
        pass
    import torch
    from ..parallel import dist as D
    from ..runtime import modules

    use_gpu = a.device == "auto" and torch.cuda.is_available()
    rank, world, device = D.init_from_env(use_gpu=use_gpu)
    if device.type == "cuda":
        from ..utils import numa
        numa.bind_to_gpu(device.index or 0)  # pinned split buffers on the GPU's socket
    n = modules.normalize
    params = {"taskfn": n(a.taskfn), "mapfn": n(a.mapfn), "partitionfn": n(a.partitionfn),
              "reducefn": n(a.reducefn), "finalfn": n(finalfn) if finalfn else None,
              "combinerfn": n(combinerfn) if combinerfn else None, "init_args": init_args,
              "checkpoint_dir": a.checkpoint_dir, "num_partitions": a.num_partitions, "result_ns": a.result_ns}
    store = None
    if a.split_glob:
        import glob
        from ..parallel.spmd import SplitStore
        files = [f for g in a.split_glob for f in sorted(glob.glob(g))]
        # each rank reads (native loader, in parallel) and pins only the
        # splits assigned to it; the engine's copies start as they land
        store = SplitStore.from_files(files, rank, world, pin=device.type == "cuda")
    from .. import spmd
    eng = spmd(params, device=device, split_store=store, verbose=a.verbose or rank == 0)
    eng.run()
    if world > 1:
        D.barrier(device=device if device.type == "cuda" else None)
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
