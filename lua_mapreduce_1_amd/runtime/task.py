"""Task singleton + job claiming (reference: mapreduce/task.lua).

The task document (``_id="unique"`` of the reference) lives in the
coordinator's per-database task map; map/reduce job documents in its job
collections.  ``take_next_job`` claims a job with ONE atomic coordinator op
(the reference's update-then-find race, task.lua:294-309, is gone) and keeps
the iteration affinity of task.lua:277-293: from iteration 2 on a worker first
asks for map jobs it executed before (data locality), and only after
``MAX_IDLE_COUNT`` idle polls for any job.
"""
from __future__ import annotations

import json
import os

from .. import utils
from ..utils import STATUS, TASK_STATUS

_VERSION = "0.4"
_NAME = "task"

TASK_FIELDS = ("status", "mapfn", "reducefn", "partitionfn", "combinerfn", "init_args", "storage", "iteration",
               "started_time", "finished_time", "stats", "device", "extra")


def tmpname_summary(tmpname: str) -> str:
    return os.path.basename(tmpname)


class task:  # noqa: N801
    # iteration-affinity cache shared by the workers of a process (task.lua:249-254)
    cache_map_ids: list[str] = []
    cache_inv_map_ids: set[str] = set()
    count_idle_iterations = 0

    def __init__(self, cnn):
        self.claimed_or_waited = False
        self.version = -1
        self.cnn = cnn
        dbname = cnn.get_dbname()
        self.ns = dbname + ".task"
        self.map_jobs_ns = "map_jobs"
        self.map_results_ns = "map_results"
        self.red_jobs_ns = "red_jobs"
        self.red_results_ns = "red_results"
        self.tbl: dict | None = None
        self.current_jobs_ns = None
        self.current_results_ns = None
        self.current_fname = None
        self.current_args = None

    # -- private ---------------------------------------------------------------
    def _set_status_local(self, status, tbl=None):
        self.tbl = tbl if tbl is not None else (self.tbl or {})
        self.tbl["status"] = status
        if status == TASK_STATUS.MAP:
            self.current_jobs_ns = self.map_jobs_ns
            self.current_results_ns = self.map_results_ns
            self.current_fname = self.tbl.get("mapfn")
            self.current_args = self.tbl.get("init_args")
        elif status == TASK_STATUS.REDUCE:
            self.current_jobs_ns = self.red_jobs_ns
            self.current_results_ns = self.red_results_ns
            self.current_fname = self.tbl.get("reducefn")
            self.current_args = self.tbl.get("init_args")

    def _set_fields(self, **fields):
        args = []
        for k, v in fields.items():
            args += [k, json.dumps(v)]
        self.cnn.connect().request("TASK_SET", self.cnn.get_dbname(), *args)

    # -- public ------------------------------------------------------------------
    def create_collection(self, task_status, params: dict, iteration: int) -> None:
        self._set_fields(status=task_status, mapfn=params.get("mapfn"), reducefn=params.get("reducefn"),
                         partitionfn=params.get("partitionfn"), combinerfn=params.get("combinerfn"),
                         init_args=params.get("init_args"), storage=params.get("storage"), iteration=iteration,
                         device=params.get("device"), extra=params.get("extra"), started_time=0, finished_time=0)
        self.tbl = dict(params)
        self.tbl["status"] = task_status
        self.tbl["iteration"] = iteration

    def get_storage(self):
        return utils.get_storage_from(self.tbl["storage"])

    def insert_finished_time(self, t: float) -> None:
        self._set_fields(finished_time=t)

    def insert_started_time(self, t: float) -> None:
        self._set_fields(started_time=t)

    def insert(self, t: dict) -> None:
        self._set_fields(**t)

    def update(self) -> None:
        st, f = self.cnn.connect().request("TASK_GET", self.cnn.get_dbname())
        tbl = {f[i].decode(): json.loads(f[i + 1]) for i in range(0, len(f), 2)}
        # the coordinator's mutation count at this read (long polls wait for
        # a change after it)
        self.version = int(tbl.pop("_ver", -1))
        if st == 0:
            self._set_status_local(tbl.get("status"), tbl)
        else:
            self.tbl = None
            self.current_jobs_ns = None
            self.current_results_ns = None
            self.current_fname = None
            self.current_args = None

    def finished(self) -> bool:
        return self.tbl is None or self.tbl.get("status") == TASK_STATUS.FINISHED

    def get_task_status(self):
        return self.tbl.get("status") if self.tbl else TASK_STATUS.FINISHED

    def has_status(self) -> bool:
        return self.tbl is not None

    def get_iteration(self) -> int:
        return int(self.tbl.get("iteration") or 0)

    def set_task_status(self, status, extra: dict | None = None) -> None:
        self._set_fields(status=status)
        if extra:
            self._set_fields(**extra)
        self._set_status_local(status, self.tbl)

    def drop(self) -> None:
        self.cnn.connect().request("TASK_DROP", self.cnn.get_dbname())

    # namespace getters (task.lua:195-245)
    def get_task_ns(self):
        return self.ns

    def get_map_jobs_ns(self):
        return self.map_jobs_ns

    def get_red_jobs_ns(self):
        return self.red_jobs_ns

    def get_map_results_ns(self):
        return self.map_results_ns

    def get_red_results_ns(self):
        return self.red_results_ns

    def get_jobs_ns(self):
        return self.current_jobs_ns

    def get_results_ns(self):
        return self.current_results_ns

    def get_fname(self):
        return self.current_fname

    def get_args(self):
        return self.current_args

    def get_reduce_fname(self):
        return self.tbl.get("reducefn")

    def get_reduce_args(self):
        return self.tbl.get("init_args")

    def get_partition_fname(self):
        return self.tbl.get("partitionfn")

    def get_partition_args(self):
        return self.tbl.get("init_args")

    def get_combiner_fname(self):
        return self.tbl.get("combinerfn")

    @classmethod
    def reset_cache(cls) -> None:
        cls.cache_map_ids = []
        cls.cache_inv_map_ids = set()

    # -- job claim -------------------------------------------------------------
    def take_next_job(self, tmpname: str, worker_name: str | None = None, wait: float = 0.0):
        """Returns (task_status, job | None).  ``wait`` > 0: the last claim
        is a long poll of up to ``wait`` seconds (``claimed_or_waited`` tells
        the caller whether a claim was made at all: not while the task is in
        WAIT or FINISHED)."""
        from .job import job  # local import (job imports task-level helpers)

        self.claimed_or_waited = False
        status = self.get_task_status()
        if status in (TASK_STATUS.WAIT, TASK_STATUS.FINISHED):
            return status, None
        self.claimed_or_waited = True
        jobs = self.cnn.jobs(self.get_jobs_ns())
        worker = worker_name or utils.get_hostname()
        t = utils.time()
        claim_kwargs = {"statuses": (STATUS.WAITING, STATUS.BROKEN)}
        if self.get_iteration() > 1 and status == TASK_STATUS.MAP:
            cls = type(self)
            job_tbl = jobs.claim(worker, tmpname_summary(tmpname), t, only_ids=cls.cache_map_ids) \
                if cls.cache_map_ids else None
            if job_tbl is None:
                cls.count_idle_iterations += 1
                if cls.count_idle_iterations <= utils.MAX_IDLE_COUNT:
                    claim_kwargs = {"statuses": (STATUS.BROKEN,)}
                job_tbl = jobs.claim(worker, tmpname_summary(tmpname), t, wait=wait, **claim_kwargs)
        else:
            job_tbl = jobs.claim(worker, tmpname_summary(tmpname), t, wait=wait, **claim_kwargs)
        if job_tbl is None:
            return TASK_STATUS.WAIT, None
        type(self).count_idle_iterations = 0
        if status == TASK_STATUS.MAP and job_tbl["_id"] not in type(self).cache_inv_map_ids:
            type(self).cache_inv_map_ids.add(job_tbl["_id"])
            type(self).cache_map_ids.append(job_tbl["_id"])
        storage, path = self.get_storage()
        return status, job(self.cnn, job_tbl, status, self.get_fname(), self.get_args(), jobs, self.get_results_ns(),
                           combiner=self.get_reduce_fname(), partitioner=self.get_partition_fname(),
                           storage=storage, path=path, task_tbl=self.tbl)


def utest() -> None:
    """task.lua:365-367."""
    assert tmpname_summary("/tmp/lua_worker_abc") == "lua_worker_abc"
