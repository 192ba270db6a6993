"""SPMD engine for host-only user modules (a ``mapfn`` without ``device_mapfn``).

The same launch shape as :class:`parallel.spmd.SPMDEngine` — one process per
rank, taskfn on rank 0 (or replicated), map jobs in contiguous blocks per
rank, partition ``p`` owned by rank ``p % W``, finalfn on rank 0, ``"loop"``,
checkpoint/resume and fault injection — with the reference's host semantics
for everything the user writes in Python:

* map: ``mapfn(key, value, emit)`` groups values by key, the combiner fires
  when a key holds more than ``MAX_MAP_RESULT`` values and once per key at the
  end of the job (job.lua:92-96, 154-228); ``partitionfn(key)`` must return an
  integer (job.lua:200-206);
* shuffle: every rank's (partition -> key -> values) pieces go to the owning
  rank in one object all-to-all (there is no shared storage to spill to);
* reduce: keys in the reference's total order (utils.lua:123-128), values
  concatenated in job order, ``reducefn(key, values, emit)`` skipped for a
  single value when the reducer is associative+commutative+idempotent
  (job.lua:253-296); results named ``<result_ns>.P<NN>`` and handed to finalfn
  sorted by name (server.lua:358-383).

It lets ``execute_spmd`` run any reference-style module; the word-count data
plane (device_mapfn) keeps using the HIP kernels through SPMDEngine.
"""
from __future__ import annotations

import sys
import time
import traceback

from .. import utils
from ..runtime import codec, modules
from ..utils import STATUS
from ..utils.tuple import tuple as tuple_
from . import dist as D
from .spmd import IterationResult, JobRecord, SPMDEngine, assign_contiguous


class HostSPMDEngine(SPMDEngine):
    def __init__(self, params: dict, group=None, device=None, verbose: bool = False, **_ignored):
        import torch
        self.params = dict(params)
        self.group = group
        self.rank, self.world = D.world_info(group)
        self.device = torch.device(device or "cpu")
        self.splits = None
        self.verbose = verbose
        self.result_ns = self.params.get("result_ns") or "result"
        self.init_args = self.params.get("init_args")
        self.taskfn = modules.load(self.params["taskfn"])
        self.mapmod = modules.load(self.params["mapfn"])
        self.partmod = modules.load(self.params["partitionfn"])
        self.redmod = modules.load(self.params["reducefn"])
        self.finalmod = modules.load(self.params.get("finalfn")) if self.params.get("finalfn") else None
        cname = self.params.get("combinerfn")
        self.combmod = modules.load(cname) if cname else None
        seen: set = set()
        for m in (self.taskfn, self.mapmod, self.partmod, self.redmod, self.finalmod, self.combmod):
            # every engine is a new task: its modules' inits run with ITS init
            # args (once per distinct init function), whatever earlier engines
            # of this process did
            modules.init_once(m, self.init_args, seen)
        self.device_input = None
        self.iteration = 0
        self.finished = False
        self.checkpoint_dir = self.params.get("checkpoint_dir") or utils_tunable_ckpt()
        self.resumed_from = 0

    # -- one iteration ------------------------------------------------------------
    def _map_job(self, key, value, combiner, partitioner) -> dict:
        result: dict = {}
        max_res = utils.MAX_MAP_RESULT

        def combine(k, values):
            out = []
            combiner(k, values, out.append)
            values[:] = [tuple_(v) for v in out]

        def emit(k, v):
            k, v = tuple_(k), tuple_(v)
            lst = result.get(k)
            if lst is None:
                result[k] = lst = []
            lst.append(v)
            if combiner is not None and len(lst) > max_res:
                combine(k, lst)

        modules.field(self.mapmod, "mapfn")(key, value, emit)
        parts: dict = {}
        for k in utils.keys_sorted(result):
            values = result[k]
            if len(values) > 1 and combiner is not None:
                combine(k, values)
            p = partitioner(k)
            try:
                pi = int(p)
            except (TypeError, ValueError):
                raise ValueError("Partition key must be a number")
            if pi != p:
                raise ValueError("Partition key must be an integer")
            parts.setdefault(pi, {})[k] = values
        return parts

    def run_iteration(self, prefetch_next=None, lookahead=None) -> IterationResult:
        self.iteration += 1
        res = IterationResult()
        T = res.timings
        t_start = time.time()
        jobs = self._jobs()
        j0, j1 = assign_contiguous([1] * len(jobs), self.rank, self.world)
        # the reducefn module's combinerfn, as the workers use (task.lua:325,
        # job.lua:160-161; runtime/job.py), else the configured combinerfn module's
        combiner = modules.field(self.redmod, "combinerfn") or (
            modules.field(self.combmod, "combinerfn") if self.combmod is not None else None)
        partitioner = modules.field(self.partmod, "partitionfn")
        local: dict = {}  # partition -> key -> values, in job order
        failed = 0
        for j in range(j0, j1):
            r = JobRecord(*jobs[j])
            r.worker, r.started = self.rank, time.time()
            c0 = time.process_time()
            for attempt in range(utils.MAX_JOB_RETRIES):
                try:
                    parts = self._map_job(r.key, r.value, combiner, partitioner)
                    break
                except Exception:  # BROKEN -> retried; FAILED after MAX_JOB_RETRIES (server.lua:194-213)
                    r.repetitions += 1
                    parts = None
                    sys.stderr.write("# rank %d map job %r attempt %d failed:\n%s" % (
                        self.rank, r.key, attempt + 1, traceback.format_exc()))
            if parts is None:
                r.status = STATUS.FAILED
                failed += 1
            else:
                r.status = STATUS.WRITTEN
                for p, kv in parts.items():
                    dst = local.setdefault(p, {})
                    for k, v in kv.items():
                        dst.setdefault(k, []).extend(v)
            r.written = time.time()
            r.cpu_time, r.real_time = time.process_time() - c0, r.written - r.started
            res.map_jobs.append(r)
        t_map = time.time()
        if self.world > 1:
            local, failed = self._shuffle_host(local, failed)
        t_shuf = time.time()
        red = modules.field(self.redmod, "reducefn")
        aci = all(bool(modules.field(self.redmod, f)) for f in
                  ("associative_reducer", "commutative_reducer", "idempotent_reducer"))
        allp = D.gather_objects(max(local) if local else -1, 0, self.group) if self.world > 1 else [
            max(local) if local else -1]
        pmax = max(allp) if self.rank == 0 else 0
        if self.world > 1:
            pmax = D.broadcast_object(pmax, 0, self.group)
        digits = len(str(max(pmax, 0)))
        self._host_parts = {}
        failed_red = 0
        for p in sorted(local):
            c0, t0 = time.process_time(), time.time()
            r = JobRecord(p, {"result": ("%s.P%0" + str(digits) + "d") % (self.result_ns, p)})
            r.worker, r.started = self.rank, t0
            recs = None
            # a reduce job that raises is BROKEN and re-run; after
            # MAX_JOB_RETRIES it is FAILED and its partition is dropped
            # (server.lua:194-213, job.lua:322-342)
            for attempt in range(utils.MAX_JOB_RETRIES):
                try:
                    recs = self._reduce_partition(local[p], red, aci)
                    break
                except Exception:  # noqa: BLE001
                    r.repetitions += 1
                    sys.stderr.write("# rank %d reduce job P%d attempt %d failed:\n%s" % (
                        self.rank, p, attempt + 1, traceback.format_exc()))
            r.written = time.time()
            r.cpu_time, r.real_time = time.process_time() - c0, r.written - t0
            if recs is None:
                r.status = STATUS.FAILED
                failed_red += 1
            else:
                r.status = STATUS.WRITTEN
                res.result_names[p] = r.value["result"]
                self._host_parts[p] = recs
            res.red_jobs.append(r)
        if self.world > 1:
            failed_red = D.all_reduce_sum_int(failed_red, self.device)
        res.failed_reduces = failed_red
        res.failed_maps = failed
        res.distinct_keys = sum(len(v) for v in self._host_parts.values())
        t_end = time.time()
        T.update(map=t_map - t_start, shuffle=t_shuf - t_map, reduce=t_end - t_shuf, iteration=t_end - t_start)
        return res

    def _shuffle_host(self, local: dict, failed: int):
        """Partition p -> rank p % W.  Each destination's partitions are
        serialised once (data-only MRK1 records, runtime/codec.py, with the
        failed-map count riding along) and exchanged by ONE byte all-to-all
        (the reference moves map_results.P<p>.M<m> files through GridFS / scp
        / a shared FS, fs.lua:141-181).  Returns (this rank's partitions,
        job-wide failed maps)."""
        send = [[(-1, [failed])] for _ in range(self.world)]
        for p, kv in local.items():
            send[p % self.world].append((p, list(kv.items())))
        recv = D.all_to_all_bytes([codec.encode_records(r) for r in send], self.device, self.group)
        mine: dict = {}
        failed = 0
        for piece in recv:  # rank order = job order: values stay in job order
            for p, kv in codec.decode_records(piece):
                if p < 0:
                    failed += int(kv[0])
                    continue
                dst = mine.setdefault(p, {})
                for k, v in kv:  # (msgpack arrays come back as tuples: hashable, equal by value)
                    lst = dst.get(k)
                    if lst is None:
                        dst[k] = list(v)
                    else:
                        lst.extend(v)
        return mine, failed

    @staticmethod
    def _reduce_partition(kv: dict, red, aci: bool) -> list:
        recs = []
        for k in utils.keys_sorted(kv):
            v = kv[k]
            if not aci or len(v) > 1:
                out = []
                red(k, v, out.append)
                v = [tuple_(x) for x in out]
            recs.append((k, v))
        return recs

    def gather_results(self, res: IterationResult) -> list:
        mine = [(res.result_names[p], self._host_parts[p]) for p in res.result_names]
        if self.world > 1:
            allp = D.gather_objects(mine, 0, self.group)
            if self.rank != 0:
                return []
            mine = [x for lst in allp for x in lst]
        return sorted(mine, key=lambda t: t[0])

    def pairs(self, gathered):
        for _name, recs in gathered:
            yield from recs


def utils_tunable_ckpt():
    from ..utils.config import TUNABLES
    return TUNABLES.spmd_checkpoint or None
