"""SPMD MapReduce engine: one rank per GPU, HBM-resident data plane, RCCL shuffle.

This is the MI355X-first execution mode of the same user contract as the
server/worker roles (taskfn / mapfn / partitionfn / reducefn / finalfn,
``map_results`` -> ``result.P<NN>`` layout, iterative ``"loop"``), designed for
throughput instead of a MongoDB-mediated job queue:

* rank 0 runs ``taskfn`` and broadcasts the job list; map jobs are assigned to
  ranks in contiguous byte-balanced blocks (P1 data parallelism);
* inputs are staged host(pinned) -> HBM on a copy stream in growing chunks
  while the map kernels consume the previous chunk on the compute stream;
* map + combine run in one per-rank HBM hash table across all the rank's jobs
  (P3 map-side combining, the combiner fused into the table);
* the shuffle is partition -> destination rank ``p % W``, a radix pack by
  destination and two ``all_to_all_single`` calls (counts, then payload) over
  RCCL/xGMI (P2);
* each rank reduces the partitions it owns in a second hash table, sorts them
  by (partition, key) and writes ``result.P<NN>`` columnar files to host memory;
* ``finalfn`` runs on rank 0 over the gathered, filename-sorted results; a
  ``"loop"`` reply starts the next iteration with the inputs still resident
  (P4/P6).

Per-job status (WAITING/RUNNING/WRITTEN/BROKEN/FAILED, repetitions) and the
reference's statistics block are kept in process; a map chunk that raises is
retried up to ``MAX_JOB_RETRIES`` times and then marked FAILED (server.lua
semantics), with the failure flag agreed across ranks before the shuffle.
"""
from __future__ import annotations

import os
import sys
import time
import traceback

import numpy as np
import torch

from .. import ops, utils
from ..utils.config import TUNABLES
from ..runtime import device as devmod
from ..runtime import modules
from ..utils import STATUS
from ..utils import trace
from . import dist as D
from .checkpoint import CheckpointMixin
from .splits import SplitStore, WindowedSplitStore, _file_pads, assign_contiguous  # noqa: F401  (public here too)
from .staging import N_ARENAS, StagingMixin

# largest map table the sparsity rule asks for (2^25 slots = 1.3 GB of HBM)
_MAX_SPARSE_CAP = 1 << 25
_BIG_TABLE = 1 << 24  # (slots) map tables this large shrink to their fit from 2x it, not 4x


def _tensor_ops() -> tuple:
    from .tensor_plane import TENSOR_OPS
    return TENSOR_OPS


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_STREAMS: dict = {}


def _engine_streams(device):
    """(copy stream, [two compute streams]) of a device, shared by every
    engine of the process.  torch hands out pool streams round-robin and the
    runtime maps them onto GPU_MAX_HW_QUEUES (4) hardware queues: a second
    engine with fresh streams (the benchmark's cold-start engine, then the
    steady-state one) landed its copy stream on a queue shared with a compute
    stream, which serialised copies behind kernels (+0.5 ms per step)."""
    if device.type != "cuda":
        return None, [None, None]
    st = _STREAMS.get(device)
    if st is None:
        st = _STREAMS[device] = (torch.cuda.Stream(device), [torch.cuda.Stream(device), torch.cuda.Stream(device)])
    return st[0], list(st[1])


class JobRecord:
    __slots__ = ("key", "value", "status", "repetitions", "started", "written", "cpu_time", "real_time", "worker")

    def __init__(self, key, value):
        self.key, self.value = key, value
        self.status = STATUS.WAITING
        self.repetitions = 0
        self.started = self.written = 0.0
        self.cpu_time = self.real_time = 0.0
        self.worker = -1


class _DeviceTimer:
    """Reusable HIP events (timing enabled) of one iteration slot: one before
    the map, one after every map chunk's launches, and the shuffle/tail
    boundaries.  Read after the iteration's final synchronisation."""

    def __init__(self):
        self._ev: list = []
        self.n = 0
        self.marks: dict[str, int] = {}
        self._st = None

    def _get(self, i: int):
        while len(self._ev) <= i:
            self._ev.append(torch.cuda.Event(enable_timing=True))
        return self._ev[i]

    def begin(self) -> None:
        """First event, on the current stream — which every mark of this
        iteration then uses (an iteration's map and tail are queued on one
        stream; looking the current stream up per event cost ~5 us of host
        time each)."""
        self.n = 0
        self.marks = {}
        self._st = torch.cuda.current_stream()
        self._get(0).record(self._st)

    def mark(self, name: str | None = None) -> None:
        """Event on the iteration's stream after the work queued so far."""
        self.n += 1
        self._get(self.n).record(self._st)
        if name is not None:
            self.marks[name] = self.n

    def ms(self, a: int, b: int) -> float:
        return float(self._ev[a].elapsed_time(self._ev[b]))


class IterationResult:
    def __init__(self):
        self._parts: dict[int, dict] | None = {}  # partition -> columnar host arrays (built on first use)
        self._cols = None
        self.result_names: dict[int, str] = {}
        self.map_jobs: list[JobRecord] = []
        self.red_jobs: list[JobRecord] = []
        self.timings: dict[str, float] = {}
        self.distinct_keys = 0
        self._vals = None
        self.bytes_shuffled = 0     # payload bytes this rank sent in the all-to-all
        self.bytes_shuffled_remote = 0  # ... to other ranks

    def _fresh(self) -> None:
        """The result columns of the fold plane alias the process's pinned
        download buffers (no copy per iteration); a later tail — the next
        iteration, or another engine — overwrites them.  Reading them after
        that raises instead of returning another iteration's data.  Columns
        still landing (the lazy download of an unfused tail) are waited for."""
        g = getattr(self, "_gen", None)
        if g is not None and g != devmod.pool_generation() and self._parts is None:
            raise RuntimeError("this iteration's result columns were overwritten by a later device tail: read "
                               "them (partitions, gather_results, total_value) before the next iteration runs")
        self.wait()

    def wait(self) -> None:
        """Block until this iteration's result columns are in host memory
        (they may still be landing from the device when run_iteration returns)."""
        dl = getattr(self, "_dl", None)
        if dl is not None:
            dl.wait()
            self._dl = None

    @property
    def partitions(self) -> dict[int, dict]:
        if self._parts is None:
            self._fresh()
            # copies: the partitions outlive the pinned buffers they came from
            self._parts = {p: {k: (None if v is None else np.array(v)) for k, v in
                               devmod.partition_slice(self._cols, p).items()} for p in self.result_names}
        return self._parts

    @property
    def total_value(self) -> int:
        """Sum of all reduced values of this rank (computed on first use)."""
        if getattr(self, "_total", None) is None:
            self._fresh()
            v = self._vals
            self._total = int(v.sum()) if v is not None and v.size else 0
        return self._total


class SPMDEngine(StagingMixin, CheckpointMixin):
    def __init__(self, params: dict, group=None, device=None, split_store: SplitStore | None = None,
                 chunk_mb: tuple = (2, 8, 32), verbose: bool = False, table_capacity: int = 1 << 20,
                 tail_mb: tuple = (8, 2)):
        self.params = dict(params)
        self.group = group
        self.rank, self.world = D.world_info(group)
        if device is None:
            device = devmod.default_device()
        self.device = torch.device(device)
        self.splits = split_store
        self.chunk_bytes = [int(c * (1 << 20)) for c in chunk_mb]
        # the last chunks shrink again so the kernel that runs after the final
        # H2D copy is short (the map is copy-bound on one PCIe link)
        self.tail_bytes = [int(c * (1 << 20)) for c in tail_mb]
        self.verbose = verbose
        self.result_ns = self.params.get("result_ns") or "result"
        self.init_args = self.params.get("init_args")
        self.taskfn = modules.load(self.params["taskfn"])
        self.mapmod = modules.load(self.params["mapfn"])
        self.partmod = modules.load(self.params["partitionfn"])
        self.redmod = modules.load(self.params["reducefn"])
        self.finalmod = modules.load(self.params.get("finalfn")) if self.params.get("finalfn") else None
        seen: set = set()
        for m in (self.taskfn, self.mapmod, self.partmod, self.redmod, self.finalmod):
            # every engine is a new task: its modules' inits run with ITS init
            # args (once per distinct init function), whatever earlier engines
            # of this process did
            modules.init_once(m, self.init_args, seen)
        # the reduce module's device_reduce names what the device does with a
        # key's values; WITHOUT one, nothing is folded with an op the user
        # did not declare: values are grouped on the device and the module's
        # reducefn runs per key (parallel/generic.py)
        self.op = modules.field(self.redmod, "device_reduce", None)
        spec = modules.field(self.partmod, "device_partition")
        self.nparts = int(self.params.get("num_partitions") or (spec[1] if spec else 0) or self.world)
        self.device_input = modules.field(self.mapmod, "device_input")
        self.dmap = modules.field(self.mapmod, "device_mapfn")
        if self.dmap is None:
            raise ValueError("SPMD engine needs a map module with device_mapfn (use server/worker for host-only "
                             "map functions)")
        # one map table per input slot: with pipelining, iteration i+1 maps into
        # tables[1-s] while iteration i's shuffle/reduce still reads tables[s]
        self._table_capacity = table_capacity
        self._initial_capacity = table_capacity
        # list- and record-valued reduces run on their own data planes
        # (parallel/planes.py); the fold plane below is the hash table
        from . import planes
        from ..ops import agg as _agg
        self.plane = None
        self.tables: list = [None, None]
        if self.op is None or _agg.is_column_spec(self.op) or (
                self.params.get("plane") == "generic" and self.op not in planes.RECORD_OPS):
            # (param plane="generic": the general plane also for fold / list
            # ops, e.g. to check the fused planes against it)
            self.plane_kind = "generic"
        elif self.op in planes.LIST_OPS:
            self.plane_kind = "list"
        elif self.op in planes.RECORD_OPS:
            self.plane_kind = "records"
        elif self.op in planes.FOLD_OPS:
            self.plane_kind = "fold"
            self.tables[0] = ops.HashTable(table_capacity, device=self.device, op=self.op)
        elif self.op in _tensor_ops():
            self.plane_kind = "tensor"  # dense fp32 vectors per key (parallel/tensor_plane.py)
        else:
            known = planes.FOLD_OPS + planes.LIST_OPS + planes.RECORD_OPS + _tensor_ops()
            raise ValueError(f"unknown device_reduce {self.op!r}: one of {known}, a column spec such as "
                             "'f64:sum' or ('f64:mean', 'count'), or none (the reducefn runs on the host over "
                             "device-grouped values)")
        self.red_table: ops.HashTable | None = None
        # input arenas, used round-robin by iteration sequence number q: while
        # iteration q maps/reduces arenas[q % 3], the copies of q+1 and q+2
        # (prefetch, up to two ahead) fill the other two, so the copy engine
        # streams without pause; tables and streams alternate by q % 2
        self.arenas: list = [None] * N_ARENAS
        self.slot = 0   # arena of the iteration being run / issued
        self.tslot = 0  # its table and stream
        self._seq = 0   # sequence number of the next iteration
        self._inflight: dict = {}  # arena slot -> plan key of copies issued ahead
        # HBM-resident input (P6 locality, SURVEY.md §2.5: "data stays in HBM"):
        # an arena that already holds an iteration's splits is not copied again
        self.resident = False
        self._arena_holds: dict = {}  # arena slot -> plan key of the splits it holds
        self.prefetch = False
        # build and prime the copy plans of every arena on first use (absorbs
        # one-time runtime set-up before timed iterations); off for a cold,
        # single-iteration run, where it would only add copies
        self.prime_plans = True
        self.force_shuffle = bool(self.params.get("force_shuffle", TUNABLES.force_shuffle))
        if self.force_shuffle and self.world == 1 and not D.initialized():
            raise RuntimeError("force_shuffle at world size 1 needs an initialised process group")
        if self.plane_kind != "fold":
            self.plane = planes.make_plane(self)
        # iteration pipelining (needs prefetch): the next iteration's map is
        # queued on the other slot's stream as soon as this map has finished,
        # and runs while this iteration shuffles, reduces and downloads
        self.pipeline = False
        self._pending = None
        self._rec_tmpl = None
        self.copy_stream, self.streams = _engine_streams(self.device)
        self._plans: dict = {}
        # per slot (pipelined iterations alternate): device event timers, the
        # job ranges of the map chunks and their device error words
        self._timers: list = [None, None]
        self._chunks: list = [[], []]
        self._errs: list = [None, None]
        self.iteration = 0
        self.finished = False
        # iteration manifest: rank 0 records every iteration
        # whose finalfn asked for another one, so a relaunched job (torchrun
        # --max-restarts after a rank died and tore the communicator down)
        # resumes there instead of at iteration 1
        self.checkpoint_dir = self.params.get("checkpoint_dir") or TUNABLES.spmd_checkpoint or None
        self.resumed_from = 0
        self.maps_restored = 0  # iterations whose map this rank restored from its checkpoint
        self._restored_src = None


    # ------------------------------------------------------------------------
    def _log(self, msg: str) -> None:
        if self.verbose and self.rank == 0:
            sys.stderr.write(msg)
            sys.stderr.flush()

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _jobs(self) -> list[tuple]:
        jobs = []
        # a taskfn declared pure (``spmd_replicated_taskfn = True``: its job list
        # depends only on init args) is evaluated by every rank: no broadcast —
        # and once per engine: pipelined iterations reuse the job list anyway
        replicated = bool(modules.field(self.taskfn, "spmd_replicated_taskfn"))
        if replicated and getattr(self, "_jobs_cache", None) is not None:
            return self._jobs_cache
        if self.rank == 0 or replicated:
            seen = set()

            def emit(k, v):
                if k in seen:
                    raise ValueError(f"Duplicate key: {k}")
                seen.add(k)
                jobs.append((k, v))
            modules.field(self.taskfn, "taskfn")(emit)
        if self.world > 1 and not replicated:
            jobs = D.broadcast_object(jobs, 0, self.group, self.device if self.device.type == "cuda" else None)
        if replicated:
            self._jobs_cache = jobs
        return jobs

    def _job_bytes(self, value) -> int:
        if self.device_input == "split":
            return self.splits.size(int(value["split"] if isinstance(value, dict) else value))
        if self.device_input == "file":
            import os
            return os.path.getsize(value) + 1
        if self.device_input == "records" and self.splits is not None:
            return self.splits.size(int(value["block"] if isinstance(value, dict) else value))
        return 1

    def _assign(self, jobs: list[tuple]) -> tuple[int, int]:
        """Contiguous block of jobs for this rank, balanced by input bytes
        (memoised for the cached job list of a pure taskfn)."""
        if self.world == 1:
            return 0, len(jobs)
        memo = getattr(self, "_assign_memo", None)
        if memo is not None and memo[0] is jobs:
            return memo[1]
        r = assign_contiguous([self._job_bytes(v) for _, v in jobs], self.rank, self.world)
        self._assign_memo = (jobs, r)
        return r

    # -- map ------------------------------------------------------------------
    @property
    def arena(self):
        return self.arenas[self.slot]

    @property
    def table(self) -> ops.HashTable:
        t = self.tables[self.tslot]
        if t is None:
            t = self.tables[self.tslot] = ops.HashTable(self._table_capacity, device=self.device, op=self.op)
        return t

    @table.setter
    def table(self, t: ops.HashTable) -> None:
        self.tables[self.tslot] = t

    def _fresh_table(self) -> None:
        """An empty map table for the map about to be issued: the slot's table
        reset, or replaced by a larger one once an earlier map's distinct-key
        count has raised the target capacity (``_map_sync``)."""
        t = self.tables[self.tslot]
        shrink = 2 if self._table_capacity >= _BIG_TABLE else 4  # (as _adapt_capacity)
        if t is not None and (t.cap < self._table_capacity or t.cap >= shrink * self._table_capacity):
            self.tables[self.tslot] = t = None  # grown, or far too large (every tail scans each slot)
        if t is None:
            self.tables[self.tslot] = ops.HashTable(self._table_capacity, device=self.device, op=self.op)
        else:
            t.reset()

    def _use(self, q: int) -> None:
        """Make iteration q's arena, table and stream current."""
        self.slot, self.tslot = q % N_ARENAS, q % 2

    def _timer(self):
        """The device timer of the current slot (None: timing off / CPU)."""
        if not (TUNABLES.device_timing and self.device.type == "cuda"):
            return None
        t = self._timers[self.tslot]
        if t is None:
            t = self._timers[self.tslot] = _DeviceTimer()
        return t

    def _err_words(self, n: int) -> torch.Tensor:
        """Per-chunk device error words of the current slot (zeroed here)."""
        e = self._errs[self.tslot]
        if e is None or e.numel() < n:
            e = self._errs[self.tslot] = torch.zeros(max(64, 2 * n), dtype=torch.int32, device=self.device)
        else:
            e[:n].zero_()
        return e

    def _run_map(self, jobs, recs, j0, j1) -> None:
        """Issue the map of this rank's jobs [j0, j1), chunk by chunk as the
        staged input lands.  A chunk = the jobs of one launch; its jobs share
        a device error word (``emit.error_word()``) that device code sets to
        report the chunk failed — checked after the map's synchronisation
        (``_map_sync``), which re-runs it (BROKEN) or drops it (FAILED after
        MAX_JOB_RETRIES attempts), like a host exception at launch time."""
        ctx = devmod.DeviceMapContext.__new__(devmod.DeviceMapContext)
        ctx.device, ctx.op, ctx.table = self.device, self.op, self.table
        ctx.arena, ctx.sources, ctx.base, ctx.host_pairs = None, [], 0, []
        if self.device_input == "split":
            # the staged splits ARE the key-byte source: the map reads them in
            # place (ctx.base = offset of each mapped chunk in the arena)
            ctx.sources = None
        ctx.emit = devmod.DeviceEmitter(ctx)
        self._ctx = ctx
        timer = self._timer()
        if timer is not None:
            timer.begin()
        chunks = self._chunks[self.tslot] = []
        self._mapped_bytes = 0
        errs = self._err_words(j1 - j0 + 1) if self.device.type == "cuda" else None
        fault = self._device_fault_spec()
        # the rank's whole staged input is ONE byte source (rep offsets index it)
        for (a, b), data in self._stage_chunks(jobs, j0, j1):
            k = len(chunks)
            chunks.append((a, b))
            t0 = time.time()
            c0 = time.process_time()
            if all(recs[j].status == STATUS.FAILED for j in range(a, b)):
                if timer is not None:
                    timer.mark()
                continue  # FAILED after MAX_JOB_RETRIES: left out of the results
            for j in range(a, b):
                recs[j].status, recs[j].started, recs[j].worker = STATUS.RUNNING, t0, self.rank
            keys = [jobs[j][0] for j in range(a, b)]
            if isinstance(data, torch.Tensor):
                self._mapped_bytes += data.numel()
            ctx.err_word = errs[k:k + 1] if errs is not None else None
            ctx.chunk = data if isinstance(data, torch.Tensor) else None
            done = False
            while not done:
                try:
                    if isinstance(data, torch.Tensor) and self.device_input == "split" and self.arena is not None:
                        # rep offsets relative to the arena start
                        base = data.data_ptr() - self.arena.data_ptr()
                        ctx.base = base
                        ctx.arena = self.table.src = self.arena
                        self.dmap(keys if b - a > 1 else keys[0], data, ctx.emit)
                    else:
                        self.dmap(keys[0] if b - a == 1 else keys, data, ctx.emit)
                    done = True
                except Exception:  # noqa: BLE001
                    for j in range(a, b):
                        recs[j].repetitions += 1
                        recs[j].status = STATUS.BROKEN
                    sys.stderr.write("Error executing a job: %s\n" % traceback.format_exc())
                    if recs[a].repetitions >= utils.MAX_JOB_RETRIES:
                        for j in range(a, b):
                            recs[j].status = STATUS.FAILED
                        done = True
            if fault is not None and errs is not None and fault[0] in range(a, b) and fault[1] > 0:
                # MR_SPMD_DEVICE_FAULT: a device-side write of the chunk's error
                # word, as a kernel that detects bad input would do
                fault[1] -= 1
                errs[k:k + 1].fill_(1)
            if timer is not None:
                timer.mark()
            t1 = time.time()
            for j in range(a, b):
                if recs[j].status != STATUS.FAILED:
                    recs[j].status = STATUS.WRITTEN
                recs[j].written = t1
                recs[j].real_time = (t1 - t0) / (b - a)
                recs[j].cpu_time = (time.process_time() - c0) / (b - a)
        ctx.flush_host_pairs()

    def _device_fault_spec(self):
        """``MR_SPMD_DEVICE_FAULT=<job index>:<times>``: the map chunk holding
        that job reports a device-side failure in its first ``times`` runs
        (fault injection).  State lives per engine."""
        spec = os.environ.get("MR_SPMD_DEVICE_FAULT", "")
        if not spec:
            return None
        if getattr(self, "_dev_fault", None) is None or self._dev_fault[2] != spec:
            j, times = spec.split(":")
            self._dev_fault = [int(j), int(times), spec]
        return self._dev_fault

    def _map_sync(self, jobs, recs, j0, j1):
        """Synchronise the map phase: table fill + overflow + per-chunk device
        error words in one download.  Failed chunks are BROKEN and the map is
        re-run (FAILED chunks skipped); an overflowed table is regrown and the
        map re-run.  Returns (occupied slots, overflowed)."""
        while True:
            errs = self._errs[self.tslot]
            nch = len(self._chunks[self.tslot])
            if errs is not None and nch:
                c, e = ops.host_read_many([self.table.ctrl, errs[:nch]])
                n_claimed = int(c[0]) + int(c[32::32].sum())
                overflow = bool(c[1])
            else:
                n_claimed, overflow = self.table.stats()
                e = None
            sh = getattr(self, "_stream_heap", None)
            if sh is not None and self.arena is getattr(self, "_stream_buf", None):
                if int(ops.host_read(sh)[1]):
                    # the key heap ran out: long keys of some round still point
                    # into a ring slot that was refilled — redo the map with a
                    # heap twice as large (kept for later iterations)
                    cur = getattr(self, "_stream_heap_mb", TUNABLES.stream_heap_mb)
                    self._stream_heap_mb = 2 * cur
                    sys.stderr.write("# streaming map: long-key heap of %.0f MiB full, re-mapping with %.0f MiB\n" % (
                        cur, 2 * cur))
                    self.table.reset()
                    self._run_map(jobs, recs, j0, j1)
                    continue
            bad = [k for k in range(nch) if e is not None and e[k]]
            if bad:
                for k in bad:
                    a, b = self._chunks[self.tslot][k]
                    if all(recs[j].status == STATUS.FAILED for j in range(a, b)):
                        continue
                    for j in range(a, b):
                        recs[j].repetitions += 1
                        recs[j].status = STATUS.BROKEN
                        if recs[j].repetitions >= utils.MAX_JOB_RETRIES:
                            recs[j].status = STATUS.FAILED
                    sys.stderr.write("# map chunk of jobs %s..%s reported a device-side failure (attempt %d)\n" % (
                        jobs[a][0], jobs[b - 1][0], recs[a].repetitions))
                self.table.reset()
                self._run_map(jobs, recs, j0, j1)
                continue
            if overflow or n_claimed > self.table.cap // 2:
                # grow and redo this rank's map (results with an overflowed table
                # are unusable; after an overflow the key count is unknown — it
                # is at least the capacity — so the table grows 16x, else 4x
                # the count)
                grow = 16 if overflow else 4
                self.table = ops.HashTable(ops.next_pow2(grow * max(n_claimed, 1)), device=self.device, op=self.op)
                self._table_capacity = self.table.cap
                self._run_map(jobs, recs, j0, j1)
                continue
            self._adapt_capacity(n_claimed)
            return n_claimed, overflow

    def _adapt_capacity(self, n_claimed: int) -> None:
        """The map table capacity of the next maps, from this map's key count."""
        # a rank that maps a lot of input per iteration gets sparse tables
        # for its next maps (MR_MAP_SPARSITY slots per distinct key): fewer
        # probes, the flush's atomics and loads spread over more memory
        # lines (full corpus: map 2.43 -> 2.06 ms from 2^20 to 2^23 slots).
        # A small share keeps the table: the send-side compaction scans
        # every slot, which cost more than the map saved at W = 8
        # (profiles/r2/sparse/)
        big = getattr(self, "_mapped_bytes", 0) >= TUNABLES.map_sparse_min_mb * 2**20
        if n_claimed > self.table.cap // 2:
            # more than half full (still exact): the next maps get room
            self._table_capacity = max(self._table_capacity, ops.next_pow2(4 * n_claimed))
        if big:
            self._table_capacity = max(self._table_capacity, min(
                ops.next_pow2(TUNABLES.map_sparsity * max(n_claimed, 1)), _MAX_SPARSE_CAP))
        # a table grown 16x after an overflow can end far above the key
        # count: the next maps get one sized for it (load 1/4 - 1/2; the
        # tail's compaction reads every slot's line of every column)
        fit = max(ops.next_pow2(2 * max(n_claimed, 1)), self._initial_capacity,
                  min(ops.next_pow2(TUNABLES.map_sparsity * max(n_claimed, 1)), _MAX_SPARSE_CAP) if big else 0)
        # large tables come down to `fit` from twice it already: the reset and
        # the compaction stream every slot, and the grown table of 23 M bigram
        # keys (2^27 slots, 5.4 GB with the values) cost 2 ms of the step in
        # those two passes alone (profiles/r6/bigram/)
        if self._table_capacity >= (2 if fit >= _BIG_TABLE else 4) * fit:
            self._table_capacity = fit

    def _device_spans(self, res, recs, j0: int, j1: int) -> None:
        """Job records and timings from the slot's device events (after the
        iteration's final synchronisation): each map job gets its chunk's
        device span in proportion to its input bytes, each reduce job the
        tail's span in proportion to its keys."""
        timer = self._timers[self.tslot] if self._timer() is not None else None
        if timer is None:
            return
        chunks = self._chunks[self.tslot]
        T = res.timings
        for k, (a, b) in enumerate(chunks):
            span = timer.ms(k, k + 1) / 1000.0
            w = [self._job_bytes(res.map_jobs[j].value) for j in range(a, b)] if self.device_input == "split" \
                else [1] * (b - a)
            tot = float(sum(w)) or 1.0
            for j, x in zip(range(a, b), w):
                res.map_jobs[j].real_time = span * x / tot
        T["device_map"] = timer.ms(0, len(chunks)) / 1000.0 if chunks else 0.0
        m = timer.marks
        if "tail0" in m and "tail_end" in m:
            s_end = m.get("shuffle_end", m["tail0"])
            T["device_shuffle"] = timer.ms(m["tail0"], s_end) / 1000.0
            T["device_tail"] = timer.ms(s_end, m["tail_end"]) / 1000.0
            counts = res._cols["bounds"] if res._cols is not None else None
            if counts is not None and res.red_jobs:
                tot = float(counts[-1]) or 1.0
                for r in res.red_jobs:
                    p = int(r.key)
                    r.real_time = (T["device_shuffle"] + T["device_tail"]) * float(counts[p + 1] - counts[p]) / tot

    # -- shuffle + reduce -------------------------------------------------------
    def _source(self) -> torch.Tensor | None:
        restored = getattr(self, "_restored_src", None)
        if restored is not None:
            return restored  # a map output restored from its checkpoint: its own key bytes
        if self.device_input == "split":
            return self.arena
        return self._ctx.source()

    def _shuffle(self, hi, lo, val, rep, src, part, failed: int = 0, raw: bool = False, before_sync=None):
        """Send each key to rank part % W; returns received (hi, lo, val, rep,
        src) and sets the job-wide number of failed map jobs (this rank's count
        rides along with the count exchange instead of a separate all-reduce).

        Pack (3 launches, no sort: ops/shuffle.py) -> one count exchange (the
        only host synchronisation) -> two all_to_all_single (records, key
        bytes) -> received locations made absolute in the received blob."""
        from ..ops import shuffle as SH
        W = self.world
        if raw:
            # GPU: records and key bytes in ONE buffer of per-destination
            # segments -> one payload all-to-all; the receive-side insert
            # kernel locates records and bytes from the exchanged counts
            with trace.range("mr.pack"):
                buf, xchg = SH.pack_by_dest_combined(hi, lo, val, rep, part, W, src, extra=failed)
            with trace.range("mr.count_exchange"):
                recv = D.exchange_counts(xchg, self.group)
            if before_sync is not None:
                before_sync()  # host work that overlaps the pack and count exchange
            with trace.range("mr.count_sync"):
                send_h, recv_h = self._host_counts(xchg, recv, W)  # one host sync
            self._failed_total = sum(r[2] for r in recv_h)
            send_sz = [SH.seg_bytes(r[0], r[1]) for r in send_h]
            recv_sz = [SH.seg_bytes(r[0], r[1]) for r in recv_h]
            self._shuffled = (sum(send_sz), sum(send_sz) - send_sz[self.rank])
            with trace.range("mr.all_to_all"):
                rbuf = D.all_to_all_v(buf[:sum(send_sz)], send_sz, recv_sz, self.group)
            return rbuf, recv.view(W, 3), sum(r[0] for r in recv_h)
        rec, blob, xchg = SH.pack_by_dest(hi, lo, val, rep, part, W, src, extra=failed)
        recv = D.exchange_counts(xchg, self.group)
        both = self._host_counts(xchg, recv, W)  # one host sync
        send_h, recv_h = both
        self._failed_total = sum(r[2] for r in recv_h)
        send_rows, send_bytes = [r[0] for r in send_h], [r[1] for r in send_h]
        recv_rows, recv_bytes = [r[0] for r in recv_h], [r[1] for r in recv_h]
        sent = [32 * r + b for r, b in zip(send_rows, send_bytes)]
        self._shuffled = (sum(sent), sum(sent) - sent[self.rank])
        rrec = D.all_to_all_v(rec, send_rows, recv_rows, self.group)
        rblob = D.all_to_all_v(blob[:sum(send_bytes)], send_bytes, recv_bytes, self.group)
        rrep = SH.absolute_reps(rrec, recv_rows, recv_bytes)
        return rrec[:, 0].contiguous(), rrec[:, 1].contiguous(), rrec[:, 2].contiguous(), rrep, rblob

    @staticmethod
    def _host_counts(xchg, recv, W: int):
        """[send, recv] count rows on the host (one download + stream wait)."""
        both = torch.cat([xchg, recv]).view(2, W, 3)
        return (ops.host_read(both) if both.is_cuda else both.numpy()).tolist()

    def _fused_tail_ok(self) -> bool:
        """The fused tail kernels need a GPU, the built-in FNV-1 partitioner
        and at most 256 partitions."""
        spec = getattr(self.partmod, "device_partition", None) if self.partmod is not None else None
        return (self.device.type == "cuda" and spec is not None and spec[0] == "fnv1"
                and self.nparts <= 256 and TUNABLES.fused_tail)

    def _finalize_table(self, table, n: int, src, padded: bool = False) -> dict:
        """The fused device tail of a table: every launch and download queued
        by one native call (mr_tail_run, csrc/hip/tail.hip) — or, once a tail
        of this engine had to fall back to the exact key order (long keys in
        long runs of a shared prefix, e.g. n-grams), that order directly
        (the fused tie fix-up would fail the same way every iteration)."""
        cap = getattr(self, "_blob_cap", None)
        if getattr(self, "_exact_tail", False):
            hi, lo, val, rep, aos = table.compact((n, False), aos=True)
            return devmod.finalize_exact_device(hi, lo, val, rep, src, self.nparts, self.partmod, blob_cap=cap,
                                                aos=aos)
        return devmod.finalize_table_native(table, n, src, self.nparts, blob_cap=cap, padded=padded)

    # -- the W > 1 iteration with two host waits ------------------------------
    def _single_sync_ok(self, sh: bool, fused: bool) -> bool:
        """The fold plane's W > 1 iteration waits on the device only for the
        count exchange and the result download: the map's completion checks
        (table overflow, chunk error words) ride on the count exchange, and
        the reduce table's key count is never read before the tail is queued
        (the tail runs for a row bound; finalize_table_native(padded=True)).
        Not for restored or checkpointed maps (they need the key count
        first), streamed inputs or more than 255 partitions."""
        return (sh and fused and TUNABLES.single_sync and self.nparts <= 255 and self._restored_src is None
                and not self.checkpoint_dir and not self._arena_cap())

    def _send_bound(self) -> int:
        """Rows the send-side compaction is launched for: the table's slots on
        a first map, else the last map's key count plus a quarter (rounded to
        4096 rows, so the workspaces keep their shape across iterations; the
        round-4 rounding to 64 K had the W = 8 reduce tail sort 131 K rows for
        54 K keys); a map with more keys is flagged by the compaction and
        redone with its count."""
        est = getattr(self, "_send_est", None)
        if est is None:
            return self.table.cap
        b = est + est // 4 + 4096
        return min(self.table.cap, (b + 0xFFF) & ~0xFFF)

    def _exchange_single_sync(self, jobs, recs, j0: int, j1: int, before_sync):
        """Compaction, pack and count exchange queued straight behind the
        map's launches; ONE host wait downloads the exchanged counts together
        with this rank's map checks.  A rank whose map overflowed, reported a
        device error or outgrew the compaction's bound adds STATUS_REDO to its
        exchanged extra column; every rank sees it and the exchange is redone
        after that rank fixed its map (the map re-run of _map_sync).  Returns
        (received buffer, recv counts [W, 3] on the device, received rows,
        map key count)."""
        from ..ops import shuffle as SH
        W = self.world
        while True:
            src = self._source()
            failed = sum(1 for r in recs[j0:j1] if r.status == STATUS.FAILED)
            bound = self._send_bound()
            nch = len(self._chunks[self.tslot])
            errs = self._errs[self.tslot][:nch] if nch and self._errs[self.tslot] is not None else None
            with trace.range("mr.compact_pack"):
                # table -> per-destination segments in three launches (no dense columns)
                buf, xchg, cnt = SH.compact_pack(self.table, src, self.nparts, W, bound, extra=failed, errs=errs,
                                                 cap_bytes=getattr(self, "_send_cap_test", None),
                                                 min_bytes=getattr(self, "_send_cap_min", 0))
                self._send_cap_test = None  # (a test's one-shot: a send buffer too small)
            with trace.range("mr.count_exchange"):
                recv = D.exchange_counts(xchg, self.group)
                # the download (one launch that signals the host) is queued
                # before the next map is issued, so it runs during that
                rd = ops.host_read_begin([xchg, recv, self.table.ctrl[:2], cnt] + ([errs] if errs is not None else []))
            if before_sync is not None:
                before_sync()  # the next iteration's map: queued before this wait
                before_sync = None
            with trace.range("mr.count_sync"):
                got = rd.wait()
            send_h, recv_h = got[0].reshape(W, 3).tolist(), got[1].reshape(W, 3).tolist()
            c = got[2]
            overflow = bool(c[1])
            n_claimed = int(got[3][0])
            e = got[4] if errs is not None else None
            if not any(r[2] >= SH.STATUS_REDO for r in recv_h):
                break
            # a redo: this rank fixes what it flagged, every rank exchanges again
            self._send_est = n_claimed
            # the exchanged row holds the true per-destination totals even when
            # the send buffer was too small: the next buffer holds them all, so
            # a redo for capacity always makes progress (the floor is kept:
            # the key-byte total of overlapping keys does not shrink)
            need = sum(SH.seg_bytes(r[0], r[1]) for r in send_h)
            if need > getattr(self, "_send_cap_min", 0):
                self._send_cap_min = need + need // 8
            bad = [k for k in range(nch) if e is not None and e[k]]
            if bad:
                self._mark_broken(jobs, recs, bad)
                self.table.reset()
                self._run_map(jobs, recs, j0, j1)
            elif overflow:
                self.table = ops.HashTable(ops.next_pow2(16 * max(n_claimed, 1)), device=self.device, op=self.op)
                self._table_capacity = self.table.cap
                self._run_map(jobs, recs, j0, j1)
        self._send_est = n_claimed
        self._adapt_capacity(n_claimed)
        self._failed_total = sum(r[2] & (SH.STATUS_REDO - 1) for r in recv_h)
        send_sz = [SH.seg_bytes(r[0], r[1]) for r in send_h]
        recv_sz = [SH.seg_bytes(r[0], r[1]) for r in recv_h]
        self._shuffled = (sum(send_sz), sum(send_sz) - send_sz[self.rank])
        with trace.range("mr.all_to_all"):
            rbuf = D.all_to_all_v(buf[:sum(send_sz)], send_sz, recv_sz, self.group)
        return rbuf, recv.view(W, 3), sum(r[0] for r in recv_h), n_claimed

    def _mark_broken(self, jobs, recs, bad_chunks) -> None:
        """Chunks whose device error word was set: BROKEN (FAILED after
        MAX_JOB_RETRIES attempts), to be re-run (server.lua:194-205)."""
        for k in bad_chunks:
            a, b = self._chunks[self.tslot][k]
            if all(recs[j].status == STATUS.FAILED for j in range(a, b)):
                continue
            for j in range(a, b):
                recs[j].repetitions += 1
                recs[j].status = STATUS.BROKEN
                if recs[j].repetitions >= utils.MAX_JOB_RETRIES:
                    recs[j].status = STATUS.FAILED
            sys.stderr.write("# map chunk of jobs %s..%s reported a device-side failure (attempt %d)\n" % (
                jobs[a][0], jobs[b - 1][0], recs[a].repetitions))

    def _reduce_insert_bound(self, rbuf, recv_counts, rows: int) -> int:
        """Received records -> the reduce table WITHOUT reading its key count:
        the table is sized from the previous iteration's distinct keys (or the
        received rows), and the returned row bound — at most the received
        rows — launches the padded tail, which flags a table that overflowed
        or outgrew the bound (TailBoundError: _retry_tail)."""
        guess = getattr(self, "_red_distinct", None)
        want = 2 * (guess + guess // 4) if guess is not None else 2 * rows
        cap = ops.next_pow2(max(1 << 16, min(2 * rows, want)))
        cleared = self._wait_red_reset()
        if self.red_table is None or self.red_table.cap != cap:
            self.red_table = ops.HashTable(cap, device=self.device, op=self.op)
        elif not cleared:
            self.red_table.reset()
        self.red_table.insert_received(rbuf, recv_counts, self.world, rows=rows)
        if guess is None:
            return max(rows, 1)
        b = guess + guess // 4 + 4096
        return max(1, min(rows, (b + 0xFFF) & ~0xFFF))

    def _wait_red_reset(self) -> bool:
        """If the last padded tail queued the reduce table's reset (on its own
        stream, after its results were read), order this stream after it;
        True when that reset happened."""
        ev, self._red_reset_ev = getattr(self, "_red_reset_ev", None), None
        if ev is None:
            return False
        torch.cuda.current_stream(self.device).wait_event(ev)
        return True

    def _reduce_insert_received(self, rbuf, recv_counts, rows: int) -> int:
        """Received records -> this rank's reduce table (one insert launch);
        returns its key count.  The table is sized from the previous
        iteration's distinct-key count (its compaction scans every slot), not
        from the received rows (every peer sends the popular keys); a table
        that ends up more than half full is regrown and refilled."""
        n = rows
        guess = getattr(self, "_red_distinct", None)
        want = 2 * (guess + guess // 4) if guess is not None else 2 * n
        cap = ops.next_pow2(max(1 << 16, min(2 * n, want)))
        self._wait_red_reset()
        while True:
            if self.red_table is None or self.red_table.cap != cap:
                self.red_table = ops.HashTable(cap, device=self.device, op=self.op)
            else:
                self.red_table.reset()
            self.red_table.insert_received(rbuf, recv_counts, self.world, rows=rows)
            with trace.range("mr.reduce_sync"):
                m, ovf = self.red_table.stats()
            if not ovf and m <= cap // 2:
                self._red_distinct = m
                return m
            if cap >= ops.next_pow2(2 * n):
                if ovf:
                    raise OverflowError("reduce table overflow")
                self._red_distinct = m
                return m
            cap = ops.next_pow2(max(2 * m, 2 * cap))

    def _reduce(self, hi, lo, val, rep, src):
        n = hi.numel()
        cap = ops.next_pow2(max(1 << 16, 2 * n))
        if self.red_table is None or self.red_table.cap < cap:
            self.red_table = ops.HashTable(cap, device=self.device, op=self.op)
        else:
            self.red_table.reset()
        self.red_table.insert(hi, lo, val, rep, src=src)
        return self.red_table.compact()

    # ------------------------------------------------------------------------
    def _can_pipeline(self) -> bool:
        return (self.copy_stream is not None and self.device_input == "split" and not self._arena_cap()
                and bool(modules.field(self.taskfn, "spmd_replicated_taskfn")))

    def _issue_next_map(self, jobs, j0, j1, q: int, gate=None) -> None:
        """Queue iteration q+1's map (same job list: the taskfn is pure) on its
        own arena, table and stream, then return to iteration q's.  Its table
        and stream were last used by iteration q-1, which has fully completed
        (its results were downloaded).  ``gate``: an event the map (not the
        table reset) waits for."""
        self._prefetch(jobs, j0, j1, q + 1)
        recs = self._new_records(jobs, j0, j1)
        self._use(q + 1)
        try:
            st = self.streams[self.tslot]
            with torch.cuda.stream(st):
                self._fresh_table()
                if gate is not None:
                    st.wait_event(gate)
                t0 = time.time()
                self._run_map(jobs, recs, j0, j1)
        finally:
            self._use(q)
        self._pending = {"q": q + 1, "jobs": jobs, "recs": recs, "j0": j0, "j1": j1, "t0": t0}

    def run_iteration(self, prefetch_next: bool | None = None, lookahead: int | None = None) -> IterationResult:
        with trace.range("mr.iteration"):
            if self.plane is not None:
                return self.plane.run_iteration(prefetch_next, lookahead)
            return self._run_iteration(prefetch_next, lookahead)

    def _new_records(self, jobs, j0: int, j1: int) -> list[JobRecord]:
        """Fresh records for this rank's jobs [j0, j1); the other ranks' jobs
        share WAITING records that nothing mutates (cached per job list: a
        record per job per iteration cost ~40 us of host time at 8 ranks)."""
        tmpl = self._rec_tmpl
        if tmpl is None or tmpl[0] is not jobs:
            tmpl = self._rec_tmpl = (jobs, [JobRecord(k, v) for k, v in jobs])
        recs = list(tmpl[1])
        for j in range(j0, j1):
            recs[j] = JobRecord(*jobs[j])
        return recs

    def _run_iteration(self, prefetch_next, lookahead) -> IterationResult:
        """One MapReduce iteration.  ``prefetch_next`` (default ``self.prefetch``)
        starts the input copies of the next ``lookahead`` (default 2, at most
        N_ARENAS - 1) iterations as soon as their arenas are free; with
        ``self.pipeline`` the next iteration's map is also queued as soon as
        this map is done.  ``prefetch_next=False`` starts nothing ahead."""
        self.iteration += 1
        if prefetch_next is None:
            prefetch_next = self.prefetch
        ahead = 0 if not prefetch_next else (N_ARENAS - 1 if lookahead is None else min(lookahead, N_ARENAS - 1))
        q = self._seq
        self._seq += 1
        self._use(q)
        res = IterationResult()
        T = res.timings
        t_start = time.time()
        pending, self._pending = self._pending, None
        if pending is not None:  # this iteration's map was queued by the previous one
            assert pending["q"] == q
            jobs, recs, j0, j1, t0 = pending["jobs"], pending["recs"], pending["j0"], pending["j1"], pending["t0"]
            stream = self.streams[self.tslot]
        else:
            trace.push("mr.jobs")
            jobs = self._jobs()
            j0, j1 = self._assign(jobs)
            recs = self._new_records(jobs, j0, j1)
            trace.pop()
            # the pipeline streams also when nothing is started ahead (the last
            # warm-up step): the first timed step then launches on warm streams
            stream = self.streams[self.tslot] if self.pipeline and self._can_pipeline() else None
        res.map_jobs = recs
        self._restored_src = None
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            if pending is None:
                with trace.range("mr.table_reset"):
                    self._fresh_table()
                t0 = time.time()
                if not self._restore_map(jobs, recs, j0, j1):
                    with trace.range("mr.map.issue"):
                        self._run_map(jobs, recs, j0, j1)
            if ahead:
                self._prefetch_ahead(jobs, j0, j1, q, ahead)
            return self._finish_iteration(res, T, t_start, t0, jobs, recs, j0, j1, ahead, q)

    def _prefetch_ahead(self, jobs, j0, j1, q: int, ahead: int) -> None:
        """Copies of iterations q+1..q+ahead (their arenas are free: iterations
        up to q-1 completed).  Issued once this iteration's tail is queued —
        the host would otherwise wait for the tail there, and the copy stream
        still holds the rest of q+1's copies, so the engine does not idle."""
        trace.push("mr.prefetch")
        mapped = self._pending["q"] if self._pending is not None else q
        for k in range(1, ahead + 1):
            if q + k > mapped:  # an issued map already consumed its copies
                self._prefetch(jobs, j0, j1, q + k)
        trace.pop()

    def _finish_iteration(self, res, T, t_start, t0, jobs, recs, j0, j1, ahead, q) -> IterationResult:
        prefetch_next = ahead > 0
        pipelined = prefetch_next and self.pipeline and self._can_pipeline()
        # When the next iteration's map is queued: host-staged input —
        # right after this iteration's tail kernels (W=1) / its count exchange
        # (W>1), so those get the GPU first; HBM-resident input ("chain") —
        # before this map's synchronisation, gated on its completion by an
        # event, so two maps run back to back and the GPU never idles while
        # the host syncs and issues (the tail's short kernels run beside the
        # next map).  The other orders measured slower (profiles/r2/next_map/,
        # removed in round 3: profiles/r3/pruned/).
        next_map = [pipelined]

        def issue_next_map(gate=None):
            if next_map[0]:
                next_map[0] = False
                with trace.range("mr.map.issue_next"):
                    self._issue_next_map(jobs, j0, j1, q, gate)
        if self.resident and next_map[0]:
            gate = None
            if self.device.type == "cuda":
                # the next map starts when this one ends (two maps sharing the
                # GPU ran slower than one after the other)
                gate = torch.cuda.Event()
                gate.record()
            issue_next_map(gate)
        fused = self._fused_tail_ok()
        # the shuffle runs at W > 1, or at W = 1 with MR_FORCE_SHUFFLE (the
        # RCCL data path exercised on a single GPU: pack -> count exchange ->
        # all_to_all_single -> receive-side insert)
        sh = self.world > 1 or self.force_shuffle
        single = self._single_sync_ok(sh, fused)
        if not single:
            trace.push("mr.map.wait")
            if self._restored_src is not None:
                n_claimed, overflow = self.table.stats()
            else:
                n_claimed, overflow = self._map_sync(jobs, recs, j0, j1)  # synchronises the map phase
                self._save_map(n_claimed, overflow, recs, j0, j1)
            trace.pop()
        self._maybe_inject_fault("shuffle")
        T["map"] = time.time() - t0
        timer = self._timer()
        t1 = time.time()
        if timer is not None:
            timer.mark("tail0")
        src = self._source()
        failed = sum(1 for r in recs[j0:j1] if r.status == STATUS.FAILED)
        self._failed_total = failed
        pend = None
        padded = False
        if single:
            # two host waits per iteration: the count exchange (with the map's
            # checks) and the result download
            trace.push("mr.shuffle_reduce")
            src, rcounts, rows, n_claimed = self._exchange_single_sync(jobs, recs, j0, j1, issue_next_map)
            T["map"] = time.time() - t0
            if getattr(self, "_exact_tail", False):
                n_red = self._reduce_insert_received(src, rcounts, rows)
            else:
                n_red = self._reduce_insert_bound(src, rcounts, rows)
                padded = True
            if timer is not None:
                timer.mark("shuffle_end")
            with trace.range("mr.tail_issue"):
                pend = self._finalize_table(self.red_table, n_red, src, padded=padded)
            trace.pop()
        elif not sh and fused:
            # (issuing the next map before an exact-order tail, to run beside
            # it, measured slower: 15.05-15.21 vs 14.70-14.79 ms per bigram
            # step, profiles/r6/bigram/map_ahead/)
            pend = self._finalize_table(self.table, n_claimed, src)
            issue_next_map()
        elif sh and fused:
            # compact + FNV partition in one kernel (the send side of the shuffle)
            if overflow:
                raise OverflowError("hash table overflow")
            with trace.range("mr.compact"):
                hi, lo, val, rep, part = devmod.compact_partition(self.table, n_claimed, src, self.nparts)
        else:
            hi, lo, val, rep = self.table.compact((n_claimed, overflow))
            part = devmod.partition_of(hi, lo, rep, src, self.nparts, self.partmod)
        if sh and not single:
            trace.push("mr.shuffle_reduce")
            if fused:
                src, rcounts, rows = self._shuffle(hi, lo, val, rep, src, part, failed, raw=True,
                                                  before_sync=issue_next_map)
                n_red = self._reduce_insert_received(src, rcounts, rows)
                if timer is not None:
                    timer.mark("shuffle_end")
                with trace.range("mr.tail_issue"):
                    pend = self._finalize_table(self.red_table, n_red, src)
            else:
                hi, lo, val, rep, src = self._shuffle(hi, lo, val, rep, src, part, failed)
                hi, lo, val, rep = self._reduce(hi, lo, val, rep, src)
                part = devmod.partition_of(hi, lo, rep, src, self.nparts, self.partmod)
            trace.pop()
        T["shuffle"] = time.time() - t1
        t2 = time.time()
        unfused = pend is None
        if unfused:
            pend = devmod.finalize_device(hi, lo, val, rep, src, self.nparts, self.partmod, part=part,
                                          blob_cap=getattr(self, "_blob_cap", None))
        if timer is not None:
            timer.mark("tail_end")
        issue_next_map()

        with trace.range("mr.finalize_host"):
            for attempt in range(4):
                try:
                    cols = devmod.finalize_host(pend, self.partmod, lazy=True)
                    break
                except devmod.TailBoundError as e:
                    # the padded tail's bound was too small or its table
                    # overflowed (reduce_insert_bound guessed from the last
                    # iteration): refill with the synchronised sizing and re-run
                    # the tail with the count
                    if e.overflow:
                        self._red_distinct = None
                    n_red = self._reduce_insert_received(src, rcounts, rows) if e.overflow else \
                        self.red_table.stats()[0]
                    # the next iteration's bound guess follows the grown key
                    # count (else every later iteration fails the bound again)
                    self._red_distinct = int(n_red)
                    padded = False
                    pend = self._finalize_table(self.red_table, n_red, src)
                except devmod.BlobCapacityError as e:
                    # keys that overlap in the input (n-gram spans) need more key
                    # bytes than the input holds: redo the tail with room for them
                    # (remembered for the next iterations)
                    if attempt == 3:
                        raise
                    self._blob_cap = e.nbytes + e.nbytes // 8
                    if unfused:
                        pend = devmod.finalize_device(hi, lo, val, rep, src, self.nparts, self.partmod, part=part,
                                                      blob_cap=self._blob_cap)
                    else:
                        pend = self._finalize_table(self.red_table if sh else self.table,
                                                    n_red if sh else n_claimed, src, padded=padded)
        if padded:
            self._red_distinct = int(cols["val"].size)
            if self.device.type == "cuda":
                # the reduce table is cleared now, while the host reads the
                # results and issues the next iteration, instead of at the
                # head of the next iteration's post-map chain
                self.red_table.reset()
                self._red_reset_ev = torch.cuda.Event()
                self._red_reset_ev.record()
        if cols.get("exact_fallback"):
            self._exact_tail = True  # later iterations go straight to the exact order
        digits = len(str(max(self.nparts - 1, 0)))
        for p in range(self.nparts):
            if cols["bounds"][p + 1] > cols["bounds"][p]:
                res.result_names[p] = ("%s.P%0" + str(digits) + "d") % (self.result_ns, p)
                r = JobRecord(p, {"result": res.result_names[p]})
                r.status, r.started, r.written, r.worker = STATUS.WRITTEN, t1, time.time(), self.rank
                r.real_time = r.written - t1
                res.red_jobs.append(r)
        res.distinct_keys = int(cols["val"].size)
        res._dl = cols.pop("_downloads", None)  # still landing: IterationResult.wait()
        res._vals = cols["val"]
        res._cols, res._parts = cols, None
        res._gen = devmod.pool_generation() if self.device.type == "cuda" else None
        T["reduce"] = time.time() - t2
        T["iteration"] = time.time() - t_start
        res.failed_maps = self._failed_total
        res.bytes_shuffled, res.bytes_shuffled_remote = getattr(self, "_shuffled", (0, 0))
        self._device_spans(res, recs, j0, j1)
        return res

    # ------------------------------------------------------------------------
    def gather_results(self, res: IterationResult) -> list[tuple[str, dict]]:
        """All ranks' result partitions on rank 0, sorted by filename (the
        order server_final hands them to finalfn, server.lua:358-383)."""
        mine = [(res.result_names[p], res.partitions[p]) for p in res.partitions]
        if self.world > 1:
            allp = D.gather_objects(mine, 0, self.group)
            if self.rank != 0:
                return []
            mine = [x for lst in allp for x in lst]
        return sorted(mine, key=lambda t: t[0])

    def pairs(self, gathered):
        from ..runtime import codec
        for _name, cols in gathered:
            if "keys" in cols and "values" in cols:  # the tensor plane: (key, [array])
                for k, v in zip(cols["keys"], cols["values"]):
                    yield k, [v]
                continue
            yield from codec.iter_columnar(cols)

    def global_stats(self, res) -> dict:
        """The iteration's statistics over EVERY rank (server.lua:155-183,538-600
        aggregates over all job documents): sums of the jobs' cpu/real times,
        distinct keys, values and shuffled bytes; cluster times and server time
        = the slowest rank's.  A collective at W > 1 (one all-gather of a
        small vector): every rank must call it."""
        T = res.timings
        dev = "device_map" in T
        map_ct = T["device_map"] if dev else T.get("map", 0.0)
        red_ct = (T.get("device_shuffle", 0.0) + T.get("device_tail", 0.0)) if dev else \
            T.get("shuffle", 0.0) + T.get("reduce", 0.0)
        # other ranks' map jobs are shared WAITING records with zero times:
        # summing every record of this rank's list counts its own jobs only
        vec = [sum(x.cpu_time for x in res.map_jobs), sum(x.cpu_time for x in res.red_jobs),
               sum(x.real_time for x in res.map_jobs), sum(x.real_time for x in res.red_jobs),
               float(getattr(res, "distinct_keys", 0)), float(getattr(res, "total_value", 0) or 0),
               float(getattr(res, "bytes_shuffled", 0)), float(getattr(res, "bytes_shuffled_remote", 0)),
               map_ct, red_ct, T.get("iteration", 0.0), T.get("device_map", 0.0), T.get("device_shuffle", 0.0),
               T.get("device_tail", 0.0)]
        nsum = 8
        if self.world > 1:
            dev_t = self.device if self.device.type == "cuda" and not D._is_gloo(self.group) else torch.device("cpu")
            t = torch.tensor(vec, dtype=torch.float64, device=dev_t)
            allv = D.all_gather_tensor(t.view(1, -1), self.group).view(self.world, -1).cpu().numpy()
            vec = [float(allv[:, i].sum()) if i < nsum else float(allv[:, i].max()) for i in range(len(vec))]
        keys = ("map_cpu", "red_cpu", "map_real", "red_real", "distinct_keys", "values", "bytes_shuffled",
                "bytes_shuffled_remote", "map_cluster", "red_cluster", "server_time", "device_map",
                "device_shuffle", "device_tail")
        out = dict(zip(keys, vec))
        out["device_spans"] = dev
        out["failed_maps"] = getattr(res, "failed_maps", 0)  # global: rides on the count exchange
        out["failed_reduces"] = getattr(res, "failed_reduces", 0)
        out["ranks"] = self.world
        return out

    def stats_block(self, res: IterationResult) -> str:
        """The reference's statistics block (server.lua:555-600 keys and
        order) over every rank — a collective at W > 1 (global_stats)."""
        g = self.global_stats(res)
        ms, rs, mr, rr = g["map_cpu"], g["red_cpu"], g["map_real"], g["red_real"]
        map_ct, red_ct = g["map_cluster"], g["red_cluster"]
        lines = [
            "#   Map sum(cpu_time)     %f" % ms, "#   Reduce sum(cpu_time)  %f" % rs,
            "# Sum(cpu_time)           %f" % (ms + rs), "#   Map sum(real_time)    %f" % mr,
            "#   Reduce sum(real_time) %f" % rr, "# Sum(real_time)          %f" % (mr + rr),
            "# Sum(sys_time)           %f" % (mr + rr - ms - rs), "#   Map cluster time      %f" % map_ct,
            "#   Reduce cluster time   %f" % red_ct,
            "# Cluster time            %f" % (map_ct + red_ct),
            "# Failed maps     %d" % g["failed_maps"],
            "# Failed reduces  %d" % g["failed_reduces"],
            "# Server time %f" % g["server_time"],
        ]
        # SURVEY.md §5.5 additions: throughput, shuffle volume, device phases
        if g["server_time"] > 0 and g["values"]:
            lines.append("# Values/s (server time) %.6g" % (g["values"] / g["server_time"]))
        lines.append("# Distinct keys %d" % g["distinct_keys"])
        if g["bytes_shuffled"]:
            lines.append("# Bytes shuffled %d (to other ranks %d)" % (g["bytes_shuffled"], g["bytes_shuffled_remote"]))
        if g["device_spans"]:
            lines.append("# Device spans ms (slowest rank): map (H2D + kernels) %.3f, shuffle %.3f, tail %.3f" % (
                1e3 * g["device_map"], 1e3 * g["device_shuffle"], 1e3 * g["device_tail"]))
        if self.world > 1:
            lines.append("# Ranks %d (sums over every rank's jobs; cluster times = slowest rank)" % self.world)
        return "\n".join(lines) + "\n"

    def run(self) -> IterationResult:
        """Iterate until finalfn returns something other than "loop".  With a
        ``checkpoint_dir`` (param or MR_SPMD_CKPT) the job resumes after the
        last iteration an earlier launch finished.  User state that must
        survive a relaunch lives in a persistent_table, as in the reference;
        a crash between finalfn and the manifest write re-runs that iteration
        (finalfn is at-least-once, like the reference's restart)."""
        start = self._load_manifest()
        if start > self.iteration:
            self._log("# Resuming after iteration %d\n" % start)
            self.iteration = self.resumed_from = start
        while True:
            self._maybe_inject_fault()
            self._log("# Iteration %d\n" % (self.iteration + 1))
            res = self.run_iteration()
            self._log(self.stats_block(res))
            reply = None
            dfin = modules.field(self.finalmod, "device_finalfn") if self.finalmod is not None else None
            if dfin is not None:
                # SPMD extension: every rank sees its own (device-resident)
                # results, e.g. a collective validation of a 10 GB sort that
                # must not be gathered to one host; rank 0's reply counts
                reply = dfin(res, self)
            else:
                gathered = self.gather_results(res)
                if self.rank == 0 and self.finalmod is not None:
                    reply = modules.field(self.finalmod, "finalfn")(self.pairs(gathered))
            if self.world > 1:
                reply = D.broadcast_object(reply, 0, self.group, self.device if self.device.type == "cuda" else None)
            if reply != "loop":
                self.finished = True
                self._save_manifest(finished=True)
                self._drop_map_ckpt(self.iteration)
                return res
            self._save_manifest(finished=False)
            self._drop_map_ckpt(self.iteration)  # the iteration is recorded: its map outputs are consumed
            self._log("# LOOP again\n")
