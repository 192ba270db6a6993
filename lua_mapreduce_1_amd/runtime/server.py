"""Server role (reference: mapreduce/server.lua).

``server.new(connection_string, dbname, auth_table)``, ``configure(params)``
and ``loop()`` keep the reference's contract: taskfn emits one map job per
key, workers run map jobs, the server turns the partitions that appeared in
the map output into reduce jobs, waits for them, prints the statistics block
(server.lua:555-600, same keys) and hands a pairs iterator over the sorted
``result.*`` files to ``finalfn`` — which may return ``"loop"`` to start the
next iteration (iterative MapReduce).  Restart semantics (server.lua:469-502):
REDUCE -> redo reduce only, WAIT/MAP -> redo unfinished maps, FINISHED -> wipe.

New over the reference: leases — RUNNING jobs whose worker stopped
heart-beating for ``utils.JOB_LEASE_SECONDS`` are re-queued as BROKEN (the
reference hangs forever on a dead worker).
"""
from __future__ import annotations

import json
import re
import sys

from .. import utils
from ..utils.config import TUNABLES
from ..utils import STATUS, TASK_STATUS
from ..utils.tuple import tuple as tuple_
from . import codec, modules
from .cnn import cnn as cnn_cls
from .job import result_store
from .task import task as task_cls

_VERSION = "0.3"
_NAME = "mapreduce.server"

from .job import INDEX_PREFIX, INDEX_SEP  # noqa: E402


def count_digits(n: int) -> int:
    if n < 0:
        raise ValueError("Only valid for positive integers")
    if n == 0:
        return 1
    c = 0
    while n > 0:
        n //= 10
        c += 1
    return c


def _err(msg: str) -> None:
    sys.stderr.write(msg)
    sys.stderr.flush()


class server:  # noqa: N801
    def __init__(self, connection_string=None, dbname: str = "tmp", auth_table=None):
        self.cnn = cnn_cls(connection_string, dbname, auth_table)
        self.task = task_cls(self.cnn)
        self.configured = False
        self.finished = False
        self.quiet = False
        self.last_stats: dict = {}
        self.poll_sleep = utils.DEFAULT_SLEEP

    @classmethod
    def new(cls, connection_string=None, dbname: str = "tmp", auth_table=None) -> "server":
        return cls(connection_string, dbname, auth_table)

    def _log(self, msg: str) -> None:
        if not self.quiet:
            _err(msg)

    # ------------------------------------------------------------------------
    def configure(self, params: dict) -> None:
        params = dict(params)
        params["storage"] = "%s:%s" % utils.get_storage_from(params.get("storage"), True)
        self.result_ns = params.get("result_ns") or "result"
        for name in ("taskfn", "mapfn", "partitionfn", "reducefn"):
            if not params.get(name):
                raise ValueError("Fields taskfn, mapfn, partitionfn and reducefn are mandatory")
        scripts = {}
        for name in ("taskfn", "mapfn", "partitionfn", "reducefn", "finalfn", "combinerfn"):
            ref = params.get(name)
            if ref is None:
                continue
            mod = modules.load(ref)
            if modules.field(mod, name) is None and not (name == "mapfn" and modules.field(mod, "device_mapfn")):
                raise ValueError(f"Module {name} must return a table with the field {name}")
            if modules.field(mod, "init") is None:
                raise ValueError(f"Init function is needed: {name}")
            scripts[name] = mod
            params[name] = modules.name_of(ref) if isinstance(ref, str) or hasattr(ref, "__name__") else ref
        self.configuration_params = params
        self.init_args = params.get("init_args")
        self.taskfn = scripts["taskfn"]
        self.finalfn = scripts.get("finalfn")
        seen = set()
        for m in (self.taskfn, self.finalfn):
            f = modules.field(m, "init")
            if f is not None and id(f) not in seen:
                seen.add(id(f))
                f(self.init_args)
        self.configured = True

    # ------------------------------------------------------------------------
    def _pause(self) -> None:
        """Between two monitor passes: a long poll that returns as soon as a
        worker changes something (a claim, a written job, an error), at most
        one poll period (MR_LONG_POLL; else a plain sleep)."""
        if TUNABLES.long_poll:
            self._ver = self.cnn.wait_change(getattr(self, "_ver", -1), self.poll_sleep)
        else:
            utils.sleep(self.poll_sleep)

    def _monitor(self, ns: str):
        jobs = self.cnn.jobs(ns)
        n = jobs.count()
        while True:
            jobs.fail_broken(utils.MAX_JOB_RETRIES)
            jobs.expire(utils.time(), utils.JOB_LEASE_SECONDS)
            m = jobs.count(STATUS.WRITTEN, STATUS.FAILED)
            self._log("\r\t %6.1f %% " % (100.0 * m / n if n else 100.0))
            for e in self.cnn.get_errors():
                self._log("\nError from %s: %s\n" % (e["worker"], e["msg"]))
            if m >= n:
                break
            yield True
        self._log("\n")

    def _prepare_map(self):
        ns = self.task.get_map_jobs_ns()
        jobs = self.cnn.jobs(ns)
        jobs.remove_status(STATUS.BROKEN, STATUS.WAITING, STATUS.FINISHED, STATUS.RUNNING)
        seen = set()
        count = 0

        def emit(key, value):
            nonlocal count
            count += 1
            k = tuple_(key)
            if k in seen:
                raise ValueError(f"Duplicate key: {key}")
            seen.add(k)
            if isinstance(value, (dict, list, tuple)):
                if len(utils.tojson(value)) > utils.MAX_TASKFN_VALUE_SIZE:
                    raise ValueError("Exceeded maximum taskfn value size")
            # an already WRITTEN job of a restarted task keeps its document
            jobs.insert(utils.make_job(key, value))

        modules.field(self.taskfn, "taskfn")(emit)
        self.task.set_task_status(TASK_STATUS.MAP)
        return self._monitor(ns), count

    def _prepare_reduce(self):
        red_ns = self.task.get_red_jobs_ns()
        red = self.cnn.jobs(red_ns)
        red.remove_status(STATUS.BROKEN, STATUS.WAITING, STATUS.FINISHED, STATUS.RUNNING)
        storage, path = self.task.get_storage()
        results_ns = self.task.get_map_results_ns()
        match = re.compile("^" + re.escape(INDEX_PREFIX + path) + r"/.*P.*M.*$")
        parse = re.compile(r"^.*\.P([^.]+)\.M([^.]*)$")
        mappers: dict[int, set] = {}
        gfs = self.cnn.gridfs()
        for f in gfs.list({"filename": {"$regex": match.pattern}}, prefix=INDEX_PREFIX + path + "/"):
            name, _, host = f["filename"].partition(INDEX_SEP)
            m = parse.match(name)
            if not m:
                continue
            pk = int(m.group(1))
            mappers.setdefault(pk, set()).add(host or utils.DEFAULT_HOSTNAME)
        digits = count_digits(max(mappers) if mappers else 0)
        for pk in sorted(mappers):
            value = {"mappers": sorted(mappers[pk]), "file": f"{path}/{results_ns}.P{pk}",
                     "result": ("%s.P%0" + str(digits) + "d") % (self.result_ns, pk)}
            self.cnn.annotate_insert(red_ns, utils.make_job(pk, value))
        self.cnn.flush_pending_inserts(0)
        self.task.set_task_status(TASK_STATUS.REDUCE)
        return self._monitor(red_ns), len(mappers)

    def _drop_collections(self) -> None:
        # every coordinator endpoint (blob shards included) — server.lua:331-343
        for c in self.cnn.gridfs().shards:
            c.request("DB_DROP", self.cnn.get_dbname())

    def _final(self) -> None:
        storage, path = self.task.get_storage()
        rstore, _ = result_store(self.cnn, storage, path)
        match = "^" + re.escape(self.result_ns)
        files = sorted(f["filename"] for f in rstore.list({"filename": {"$regex": match}}))

        def pairs():
            for name in files:
                data = rstore.get(name) if hasattr(rstore, "get") else rstore.find_file(name)
                yield from codec.decode_records(data or b"")

        reply = modules.field(self.finalfn, "finalfn")(pairs()) if self.finalfn is not None else None
        remove_all = reply is True or reply == "loop"
        if reply not in ("loop", True, False, None):
            self._log("# WARNING!!! INCORRECT FINAL RETURN: %s\n" % (reply,))
        if reply == "loop":
            self._log("# LOOP again\n")
            self.cnn.jobs(self.task.get_map_jobs_ns()).drop()
            self.cnn.jobs(self.task.get_red_jobs_ns()).drop()
        else:
            self.finished = True
            self.task.set_task_status(TASK_STATUS.FINISHED)
        # (hbm storage: the coordinator holds the files' descriptors, removed
        # here like gridfs files; the workers free their arenas at task end)
        g = self.cnn.gridfs()
        for f in g.list():
            if not re.match(match, f["filename"]) or remove_all:
                g.remove_file(f["filename"])

    # ------------------------------------------------------------------------
    def loop(self) -> None:
        if not self.configured:
            raise RuntimeError("Call to server:configure(...) method is mandatory")
        it = 0
        self.finished = False
        while True:
            skip_map, initialize = False, True
            if it == 0:
                self.task.update()
                if self.task.has_status():
                    status = self.task.get_task_status()
                    if status == TASK_STATUS.REDUCE:
                        self._log("# WARNING: TRYING TO RESTORE A BROKEN TASK\n")
                        skip_map, initialize = True, False
                        self.configuration_params["storage"] = "%s:%s" % self.task.get_storage()
                    elif status == TASK_STATUS.FINISHED:
                        self._drop_collections()
                    else:
                        initialize = False
            if initialize:
                it += 1
                self.task.create_collection(TASK_STATUS.WAIT, self.configuration_params, it)
            else:
                it = self.task.get_iteration()
                self.task.create_collection(self.task.get_task_status(), self.configuration_params, it)
            self._log("# Iteration %d\n" % it)
            start_time = utils.time()
            self.task.insert_started_time(start_time)
            if not skip_map:
                self._log("# \t Preparing Map\n")
                step, map_count = self._prepare_map()
                self._log("# \t Map execution, size= %d\n" % map_count)
                for _ in step:
                    self._pause()
            map_count = self.cnn.jobs(self.task.get_map_jobs_ns()).count()
            self._log("# \t Preparing Reduce\n")
            step, _ = self._prepare_reduce()
            red_count = self.cnn.jobs(self.task.get_red_jobs_ns()).count()
            self._log("# \t Reduce execution, num_files= %d  size= %d\n" % (red_count * map_count, red_count))
            for _ in step:
                self._pause()
            end_time = utils.time()
            total_time = end_time - start_time
            self.task.insert_finished_time(end_time)
            self._report_stats(total_time)
            self._log("# \t Final execution\n")
            self._final()
            if self.finished:
                break
        storage, path = utils.get_storage_from(self.configuration_params["storage"])
        if storage == "shared":
            utils.remove(path)

    def _report_stats(self, total_time: float) -> None:
        ms = self.cnn.jobs(self.task.get_map_jobs_ns()).stats()
        rs = self.cnn.jobs(self.task.get_red_jobs_ns()).stats()
        mc, rc = ms["sum_cpu_time"], rs["sum_cpu_time"]
        mr, rr = ms["sum_real_time"], rs["sum_real_time"]
        mrt, rrt = ms["real_time"], rs["real_time"]
        fm, fr = ms["counts"][STATUS.FAILED], rs["counts"][STATUS.FAILED]
        lines = [
            "#   Map sum(cpu_time)     %f\n" % mc,
            "#   Reduce sum(cpu_time)  %f\n" % rc,
            "# Sum(cpu_time)           %f\n" % (mc + rc),
            "#   Map sum(real_time)    %f\n" % mr,
            "#   Reduce sum(real_time) %f\n" % rr,
            "# Sum(real_time)          %f\n" % (mr + rr),
            "# Sum(sys_time)           %f\n" % (mr + rr - mc - rc),
            "#   Map cluster time      %f\n" % mrt,
            "#   Reduce cluster time   %f\n" % rrt,
            "# Cluster time            %f\n" % (mrt + rrt),
            "# Failed maps     %d\n" % fm,
            "# Failed reduces  %d\n" % fr,
        ]
        for ln in lines:
            self._log(ln)
        stats = {
            "map_sum_cpu_time": mc, "red_sum_cpu_time": rc, "total_sum_cpu_time": mc + rc,
            "map_sum_real_time": mr, "red_sum_real_time": rr, "total_sum_real_time": mr + rr,
            "sum_sys_time": mr + rr - mc - rc, "map_real_time": mrt, "red_real_time": rrt,
            "total_real_time": mrt + rrt, "iteration_time": total_time, "failed_map_jobs": fm,
            "failed_red_jobs": fr,
        }
        self.last_stats = stats
        self.task.insert({"stats": stats})
        self._log("# Server time %f\n" % total_time)


def utest(connection_string=None, dbname: str = "test") -> None:
    assert count_digits(0) == 1 and count_digits(1) == 1 and count_digits(9) == 1
    assert count_digits(10) == 2 and count_digits(99) == 2 and count_digits(111) == 3
    assert count_digits(1111) == 4
    c = cnn_cls(connection_string, dbname)
    jobs = c.jobs("times")
    jobs.drop()
    jobs.insert({"_id": "a", "value": 1, "creation_time": 10})
    jobs.insert({"_id": "b", "value": 1, "creation_time": 14})
    jobs.update("a", cpu_time=1.5, written_time=16)
    jobs.update("b", cpu_time=2.5, written_time=20)
    st = jobs.stats()
    assert st["real_time"] == 20 - 10
    assert st["sum_cpu_time"] == 4.0
    jobs.drop()


def _dummy_json(x):
    return json.dumps(x)
