"""Worker role (reference: mapreduce/worker.lua).

``worker.new(connection_string, dbname, auth_table)``,
``configure(max_iter=, max_sleep=, max_tasks=)`` (unknown keys rejected) and
``execute()`` — a protected loop that polls the task document, claims jobs,
runs them, and on an exception marks the current job BROKEN, posts the
traceback to the error channel, sleeps and retries, dying after
``MAX_WORKER_RETRIES`` distinct failed jobs (worker.lua:112-138).

New over the reference:
* a heartbeat thread keeps the claimed job's lease alive, so the server can
  re-queue jobs of workers that die without raising (SIGKILL, node loss);
* GPU placement: ``configure(gpu="auto")`` (the default) gives each worker
  on a multi-GPU node its own device through a lock-file slot
  (utils/gpu_slots.py); an int pins a device, ``"none"`` leaves torch's default;
* a fault-injection hook for tests: ``MR_FAULT="map:<id>:raise[:n]"`` or
  ``"reduce:<id>:kill"`` raises (the first n times) or ``os._exit(137)``s when
  that job starts.
"""
from __future__ import annotations

import os
import sys
import tempfile
import threading
import traceback

from .. import utils
from ..utils import TASK_STATUS, gpu_slots
from ..utils.config import TUNABLES
from . import job as job_mod
from .cnn import cnn as cnn_cls
from .task import task as task_cls

_VERSION = "0.2"
_NAME = "mapreduce.worker"

_fault_counts: dict[str, int] = {}


def _maybe_inject_fault(status: str, job_id: str) -> None:
    spec = os.environ.get("MR_FAULT", TUNABLES.fault)  # read per call: tests inject faults at run time
    if not spec:
        return
    phase = "map" if status == TASK_STATUS.MAP else "reduce"
    for item in spec.split(","):
        parts = item.split(":")
        if len(parts) < 3 or parts[0] != phase or parts[1] != str(job_id):
            continue
        limit = int(parts[3]) if len(parts) > 3 else -1
        n = _fault_counts.get(item, 0)
        if limit >= 0 and n >= limit:
            continue
        _fault_counts[item] = n + 1
        if parts[2] == "kill":
            os._exit(137)
        raise RuntimeError(f"injected fault in {phase} job {job_id}")


class worker:  # noqa: N801
    def __init__(self, connection_string=None, dbname: str = "tmp", auth_table=None):
        self.cnn = cnn_cls(connection_string, dbname, auth_table)
        self.task = task_cls(self.cnn)
        fd, self.tmpname = tempfile.mkstemp(prefix="lua_worker_")
        os.close(fd)
        self.max_iter = 20
        self.max_sleep = 20
        self.max_tasks = 1
        self.current_job = None
        self.name = utils.get_hostname()
        self.verbose = True
        self.poll_sleep = utils.DEFAULT_SLEEP
        self.gpu = "auto"
        self._gpu_slot = None
        self._hb_stop = threading.Event()
        self._hb_thread = None
        self._stop = threading.Event()

    @classmethod
    def new(cls, connection_string=None, dbname: str = "tmp", auth_table=None) -> "worker":
        return cls(connection_string, dbname, auth_table)

    def configure(self, t: dict | None = None, **kw) -> None:
        t = dict(t or {}, **kw)
        allowed = {"max_iter", "max_sleep", "max_tasks", "verbose", "poll_sleep", "name", "gpu"}
        for k, v in t.items():
            if k not in allowed:
                raise ValueError(f"Unknown parameter: {k}")
            setattr(self, k, v)

    def _print(self, msg: str) -> None:
        if self.verbose:
            print(msg, flush=True)

    def __del__(self):
        try:
            os.remove(self.tmpname)
        except OSError:
            pass

    # -- heartbeat -------------------------------------------------------------
    def _heartbeat_loop(self):
        period = max(0.05, utils.JOB_LEASE_SECONDS / 4.0)
        hb_cnn = cnn_cls(self.cnn.connection_string, self.cnn.dbname)
        while not self._hb_stop.wait(period):
            j = self.current_job
            if j is not None:
                try:
                    hb_cnn.jobs(j.jobs.ns).update(j.get_id(), j.job_tbl.get("tmpname", ""), heartbeat=utils.time())
                except Exception:  # noqa: BLE001  (best effort)
                    pass

    def _start_heartbeat(self):
        if self._hb_thread is None:
            self._hb_thread = threading.Thread(target=self._heartbeat_loop, daemon=True)
            self._hb_thread.start()

    # -- main loop --------------------------------------------------------------
    def _worker_execute(self) -> None:
        self._print("# HOSTNAME %s" % self.name)
        task = self.task
        it = 0
        iter_sleep = self.poll_sleep
        ntasks = 0
        job_done = False
        long_poll = TUNABLES.long_poll
        while it < self.max_iter and ntasks < self.max_tasks and not self._stop.is_set():
            while not self._stop.is_set():
                task.update()
                status, j = task.take_next_job(self.tmpname, self.name, wait=self.poll_sleep if long_poll else 0.0)
                self.current_job = j
                if j is not None:
                    if not job_done:
                        self._print("# New TASK ready")
                    self._print("# \t Executing %s job _id: %r" % (status, j.status_string()))
                    t1 = utils.time()
                    _maybe_inject_fault(status, j.get_id())
                    elapsed = j.execute()
                    self.current_job = None
                    self._print("# \t\t Finished: %f elapsed user time, %f real time" % (elapsed, utils.time() - t1))
                    job_done = True
                else:
                    if task.finished():
                        break
                    self._print("# \t Running, waiting for new jobs...")
                    self.cnn.flush_pending_inserts(0)
                    if not long_poll:
                        utils.sleep(self.poll_sleep)
                    elif not task.claimed_or_waited:
                        # the task is not claimable yet (server preparing a phase): wait for a
                        # change after the task read
                        self.cnn.wait_change(task.version, self.poll_sleep)
                if task.finished():
                    break
            self.cnn.flush_pending_inserts()
            if job_done:
                self._print("# TASK done")
                # hbm storage: every reduce of the task has read this worker's
                # map files (the task finished): free its device arena
                from . import hbm_store
                hbm_store.release()
                it = 0
                iter_sleep = self.poll_sleep
                ntasks += 1
                job_done = False
                job_mod.reset_cache()
                task_cls.reset_cache()
            if ntasks < self.max_tasks:
                self._print("# WAITING...\tntasks: %d/%d\tit: %d/%d\tsleep: %.1f" %
                            (ntasks, self.max_tasks, it, self.max_iter, iter_sleep))
                if long_poll:  # the next task wakes the worker at once
                    self.cnn.wait_change(task.version, iter_sleep)
                else:
                    utils.sleep(iter_sleep)
                iter_sleep = min(self.max_sleep, iter_sleep * 1.5)
            it += 1

    def stop(self) -> None:
        """Ask the worker loop to return after its current job (embedding/tests)."""
        self._stop.set()

    def execute(self) -> None:
        failed: set = set()
        if self._gpu_slot is None:  # before any job touches the GPU
            self._gpu_slot = gpu_slots.place_worker(self.gpu)
        if self.gpu != "none":
            # a persistent worker brings up its device plane once, before it
            # claims anything (HIP context, kernel library, the map context
            # and reduce table it reuses across jobs), not inside its first job
            from . import device as dev_mod
            dev_mod.warm_worker()
        self._start_heartbeat()
        try:
            while True:
                try:
                    self._worker_execute()
                    break
                except (ConnectionError, OSError) as e:
                    # coordinator unreachable (e.g. the server that hosted it
                    # finished): back off like an idle poll, give up quietly
                    lost = getattr(self, "_lost", 0) + 1
                    self._lost = lost
                    if self.current_job is None and lost > self.max_iter:
                        self._print("# coordinator unreachable (%s): exiting" % e)
                        break
                    utils.sleep(min(self.max_sleep, self.poll_sleep * lost))
                    self.cnn.db = None
                    continue
                except Exception:  # noqa: BLE001
                    msg = traceback.format_exc()
                    if self.current_job is not None:
                        try:
                            self.current_job.mark_as_broken()
                        finally:
                            failed.add(self.current_job.get_id())
                        self.current_job = None
                    self.cnn.flush_pending_inserts(0)
                    self.cnn.insert_error(self.name, msg)
                    sys.stderr.write("Error executing a job: %s\n" % msg)
                    if len(failed) >= utils.MAX_WORKER_RETRIES:
                        break
                    utils.sleep(self.poll_sleep * 4)
            self._print("# Worker retries: %d" % len(failed))
            if len(failed) >= utils.MAX_WORKER_RETRIES:
                raise RuntimeError("Maximum number of retries achieved")
        finally:
            self._hb_stop.set()
            from . import hbm_store
            hbm_store.release()


def utest() -> None:
    return None
