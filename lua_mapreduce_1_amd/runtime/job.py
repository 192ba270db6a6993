"""Map / reduce job execution on a worker (reference: mapreduce/job.lua).

Host plane (any Python mapfn/reducefn): ``emit(k, v)`` groups values per key
(keys/values go through ``tuple()`` like job.lua:84), the combiner — taken
from the *reducefn* module's ``combinerfn`` as in task.lua:325 — fires when a
key exceeds ``MAX_MAP_RESULT`` values and again per key at the end; keys are
written sorted, one ``map_results.P<p>.M<m>`` file per partition.  Reduce
merges the partition's files (heap k-way merge), calls ``reducefn`` (skipping
singleton lists when the module declares all three ACI flags, job.lua:264-274)
and writes ``result.P<NN>``.

Device plane (module defines ``device_mapfn`` / ``device_reduce``): see
:mod:`.device` — the same files, in the columnar ``MRC1`` format.
"""
from __future__ import annotations

import os
import re
import time as _time

import numpy as np
import torch

from .. import utils
from ..utils import STATUS, TASK_STATUS
from ..utils.tuple import tuple as tuple_
from . import codec, device as dev, fs as fsmod, modules

_VERSION = "0.4"
INDEX_PREFIX = "__idx__"
INDEX_SEP = "\x1f"
_NAME = "job"

_cache: dict = {}

# diagnosis (tools/bench_server_worker.py --dump): every device map output and
# every device reduce's inputs (name, size, crc32) and result are also written
# to this directory, so a wrong final answer can be traced to the job and the
# stage (map kernel, transport, reduce) that produced it
_DUMP = os.environ.get("MR_DEBUG_DUMP") or None


def _dump(kind: str, name: str, blob: bytes) -> None:
    if _DUMP is None:
        return
    os.makedirs(_DUMP, exist_ok=True)
    path = os.path.join(_DUMP, f"{kind}.{os.path.basename(name)}.{os.getpid()}.{_time.monotonic_ns()}")
    with open(path, "wb") as f:
        f.write(blob)


def cached(func):
    """Memoise a 1-argument function (job.lua:42-55; used for partitionfn)."""
    local = _cache.setdefault(func, {})

    def f(key):
        try:
            return local[key]
        except KeyError:
            r = func(key)
            local[key] = r
            return r
        except TypeError:  # unhashable key
            return func(key)
    return f


def reset_cache() -> None:
    _cache.clear()
    modules.reset()


FOLD_OPS = ("sum", "min", "max", "count")
LIST_OPS = ("concat", "concat_unique")


def device_kind(task_tbl: dict | None, mod_map, mod_red=None) -> str | None:
    """Which device map a worker runs for a map module with ``device_mapfn``
    (None: the host ``mapfn``), from the reduce module's ``device_reduce``:

    * ``"fold"`` — sum/min/max/count of int64 values in the HBM table
      (runtime/device.py), columnar ``MRC1`` map outputs;
    * ``"cols"`` — a typed column spec (ops/agg.py), ``MRC2`` outputs merged
      by the device reduce;
    * ``"list"`` — no device_reduce (or a concat op): values grouped per key
      on the device, written as ``(key, [values])`` records that the reduce
      job hands to the module's own reducefn (job.lua:264-284) — never a
      fold the user did not declare;
    * ``"identity"`` (the record plane) runs in SPMD mode only: host mapfn."""
    want = (task_tbl or {}).get("device", "auto")
    if want in (False, "never", "host"):
        return None
    if modules.field(mod_map, "device_mapfn") is None:
        return None
    op = modules.field(mod_red, "device_reduce", None) if mod_red is not None else None
    if op in FOLD_OPS:
        return "fold"
    if op is None or op in LIST_OPS:
        return "list"
    from ..ops import agg as A
    if A.is_column_spec(op):
        return "cols"
    return None


def _use_device(task_tbl: dict | None, mod_map, mod_red=None) -> bool:
    return device_kind(task_tbl, mod_map, mod_red) is not None


class job:  # noqa: N801
    def __init__(self, cnn, job_tbl: dict, task_status, fname, init_args, jobs, results_ns,
                 not_executable: bool = False, combiner=None, partitioner=None, storage="gridfs", path="/tmp",
                 task_tbl: dict | None = None):
        self.cnn = cnn
        self.job_tbl = job_tbl
        self.jobs = jobs
        self.results_ns = results_ns
        self.t = utils.time()
        self.written = False
        self.task_tbl = task_tbl or {}
        self.storage, self.path = storage, path
        self.init_args = init_args
        if task_status == TASK_STATUS.MAP:
            func = "mapfn"
        elif task_status == TASK_STATUS.REDUCE:
            func = "reducefn"
        else:
            raise ValueError(f"Incorrect task_status: {task_status}")
        self.func = func
        self.fn = None
        if not not_executable:
            self.module = modules.load(fname)
            modules.init_once(self.module, init_args)
            if func == "mapfn":
                self.fn = self._prepare_map(combiner, partitioner)
            else:
                self.fn = self._prepare_reduce()

    # -- accessors ---------------------------------------------------------------
    def execute(self):
        if self.fn is None:
            raise RuntimeError("Forbidden execution of jobs here")
        return self.fn()

    def get_id(self):
        return self.job_tbl["_id"]

    def get_pair(self):
        return self.job_tbl["_id"], self.job_tbl["value"]

    def status_string(self):
        return self.get_id()

    def get_results_ns(self):
        return self.results_ns

    def heartbeat(self) -> None:
        self.jobs.update(self.get_id(), self.job_tbl.get("tmpname", ""), heartbeat=utils.time())

    def mark_as_finished(self) -> None:
        self.jobs.update(self.get_id(), self.job_tbl.get("tmpname", ""), status=STATUS.FINISHED,
                         finished_time=utils.time())

    def mark_as_written(self, cpu_time: float) -> bool:
        """False when the job is no longer ours (lease expired, or a restarted
        server re-created it): the caller must then leave its inputs alone,
        the job's new owner will consume them."""
        self.written = True
        now = utils.time()
        return self.jobs.update(self.get_id(), self.job_tbl.get("tmpname", ""), status=STATUS.WRITTEN,
                                written_time=now, cpu_time=cpu_time, real_time=now - self.t) is not None

    def mark_as_broken(self) -> None:
        if not self.written:
            self.jobs.update(self.get_id(), self.job_tbl.get("tmpname", ""), status=STATUS.BROKEN,
                             broken_time=utils.time(), inc_repetitions=1)

    # -- map -----------------------------------------------------------------------
    def _prepare_map(self, combiner_fname, partitioner_fname):
        pmod = modules.load(partitioner_fname)
        modules.init_once(pmod, self.init_args)
        partitioner = cached(modules.field(pmod, "partitionfn"))
        cmod = modules.load(combiner_fname) if combiner_fname else None
        if cmod is not None:
            modules.init_once(cmod, self.init_args)
        combiner = modules.field(cmod, "combinerfn") if cmod is not None else None
        kind = device_kind(self.task_tbl, self.module, cmod)
        host_run = self._host_map(combiner, partitioner)
        if kind is not None:
            return lambda: self._run_device_map(pmod, cmod, kind, host_run)
        return host_run

    def _host_map(self, combiner, partitioner):
        g = modules.field(self.module, "mapfn")
        map_key, map_value = self.get_pair()

        def run():
            clock1 = _time.process_time()
            result: dict = {}
            max_res = utils.MAX_MAP_RESULT

            def combine(key, values):
                out = []
                combiner(key, values, out.append)
                values[:] = [tuple_(v) for v in out]

            def emit(key, value):
                key, value = tuple_(key), tuple_(value)
                lst = result.get(key)
                if lst is None:
                    result[key] = lst = []
                lst.append(value)
                if combiner is not None and len(lst) > max_res:
                    combine(key, lst)

            g(map_key, map_value, emit)
            self.mark_as_finished()
            fs, make_builder, _ = fsmod.router(self.cnn, None, self.storage, self.path, self._gen())
            parts: dict[int, list] = {}
            for key in utils.keys_sorted(result):
                values = result[key]
                if len(values) > 1 and combiner is not None:
                    combine(key, values)
                p = partitioner(key)
                try:
                    pi = int(p)
                except (TypeError, ValueError):
                    raise ValueError("Partition key must be a number")
                if pi != p:
                    raise ValueError("Partition key must be an integer")
                parts.setdefault(pi, []).append((key, values))
            for pi, recs in parts.items():
                name = f"{self.path}/{self.results_ns}.P{pi}.M{map_key}"
                b = make_builder()
                b.append(codec.encode_records(recs))
                fs.remove_file(name)
                b.build(name)
                self._register_output(name)
            elapsed = _time.process_time() - clock1
            self.mark_as_written(elapsed)
            return elapsed
        return run

    def _gen(self):
        """The task iteration this job's outputs belong to (hbm storage:
        the arena of an earlier iteration is released by the next one)."""
        return (self.cnn.dbname, self.task_tbl.get("iteration"))

    def _register_output(self, name: str) -> None:
        """Index the file in the coordinator so the server can find partitions
        whatever the storage (sshfs files are only on the mapper's host)."""
        self.cnn.gridfs().store_data(b"", INDEX_PREFIX + name + INDEX_SEP + utils.get_hostname())

    def _run_device_map(self, pmod, rmod, kind: str = "fold", host_run=None):
        # the device plane's pinned download buffers and workspaces are
        # per-process: worker threads of one process take turns on the GPU
        from ..parallel.generic import NeedsHostMap
        try:
            with dev.PLANE_LOCK:
                if kind == "fold":
                    return self._run_device_map_locked(pmod, rmod)
                return self._run_generic_map(pmod, rmod, kind)
        except NeedsHostMap:
            # the device map needs an SPMD-only emitter (global line numbers,
            # the record plane): the module's host mapfn does this job
            if host_run is None or modules.field(self.module, "mapfn") is None:
                raise
            return host_run()

    def _run_generic_map(self, pmod, rmod, kind: str):
        """General device map of one job (parallel/generic.py): typed folds
        (``MRC2`` partition files) or per-key value lists (``MRK1`` records
        for the host reducefn)."""
        from ..ops import agg as A
        from ..parallel import generic as G
        clock1 = _time.process_time()
        map_key, map_value = self.get_pair()
        spec = modules.field(rmod, "device_reduce", None) if rmod is not None else None
        extra = self.task_tbl.get("extra") or {}
        pspec = modules.field(pmod, "device_partition")
        nparts = int(extra.get("num_partitions") or (pspec[1] if pspec else 0) or 1)
        phys = A.Physical(A.parse_spec(spec)) if kind == "cols" else None
        from ..parallel import values as VL
        dtype = VL.spec_of(modules.field(self.module, "device_value_dtype", "i64") or "i64")
        d = dev.default_device()
        cap = int(extra.get("table_capacity") or 1 << 16)
        fn = modules.field(self.module, "device_mapfn")
        # no device_reduce: the reduce module's combiner runs over the job's
        # device-grouped lists (batched, or per key on the host) before the
        # partition files are written (job.lua:92-96,198-202)
        reducers = None
        if kind == "list" and spec is None and rmod is not None:
            from ..parallel import reducers as RD
            reducers = RD.ListReducers(rmod, dtype)
        for _ in range(8):
            gm = G.GenericMap(d, cap, phys, dtype, reducers, int(extra.get("combine_postings") or 0))
            gm.begin(None)
            fn(map_key, map_value, gm.emit)
            gm.flush_host()
            n, ovf = gm.table.stats()
            if not ovf and n <= gm.table.cap // 2 + 1:
                break
            cap = ops_next_pow2(4 * max(n, 1))
        else:
            raise OverflowError("device map table overflow")
        gm.combine()
        n = gm.table.stats()[0]
        dev.STATS["maps_" + d.type] = dev.STATS.get("maps_" + d.type, 0) + 1
        self.mark_as_finished()
        src = gm.src.source()
        if kind == "cols":
            out = G.order_fold(*gm.table.compact(), src, nparts, pmod, phys, outputs=False)
        else:
            space = gm.table.cap if gm.table.is_cuda else max(1, n)
            out = G.order_lists(*gm.table.postings(), src, nparts, pmod, spec == "concat_unique", dtype, space)
        parts = G.host_partitions(out, nparts, dtype)
        host = utils.get_hostname()
        outputs, index = [], []
        for p, cols in sorted(parts.items()):
            name = f"{self.path}/{self.results_ns}.P{p}.M{map_key}"
            if kind == "cols":
                blob = codec.encode_columns(cols["hi"], cols["lo"], cols["cols"], cols["key_off"], cols["key_blob"])
            else:
                blob = codec.encode_records(codec.iter_columnar(cols))
            outputs.append((name, blob))
            index.append((INDEX_PREFIX + name + INDEX_SEP + host, b""))
        self._store_outputs(outputs, index)
        elapsed = _time.process_time() - clock1
        self.mark_as_written(elapsed)
        return elapsed

    def _store_outputs(self, outputs, index) -> None:
        """A map job's partition files and their index entries: ONE
        coordinator request for gridfs (the bytes) and hbm (descriptors of
        the bytes just copied into this worker's device arena)."""
        fs, make_builder, _ = fsmod.router(self.cnn, None, self.storage, self.path, self._gen())
        gfs = self.cnn.gridfs()
        if self.storage == "gridfs":
            gfs.store_many(outputs + index)
        elif self.storage == "hbm":
            from . import hbm_store
            gfs.store_many(hbm_store.store().put_many(outputs, self._gen()) + index)
        else:
            for name, blob in outputs:
                b = make_builder()
                b.append(blob)
                b.build(name)
            gfs.store_many(index)

    def _run_device_map_locked(self, pmod, rmod):
        clock1 = _time.process_time()
        map_key, map_value = self.get_pair()
        op = modules.field(rmod, "device_reduce")  # device_kind() checked it is a fold op
        extra = self.task_tbl.get("extra") or {}
        spec = modules.field(pmod, "device_partition")
        nparts = int(extra.get("num_partitions") or (spec[1] if spec else 0) or 1)
        ctx = dev.DeviceMapContext.for_job(op=op, capacity=int(extra.get("table_capacity") or 1 << 20))
        modules.field(self.module, "device_mapfn")(map_key, map_value, ctx.emit)
        ctx.flush_host_pairs()
        self.mark_as_finished()
        cols = dev.finalize_table(ctx.table, ctx.source(), nparts, pmod, need_keys=True)
        # every storage's build replaces an existing file (BLOB_PUT overwrites,
        # file builders rename over), so the reference's remove-before-build
        # (job.lua:217-221) is one round trip per file with no effect; with the
        # coordinator blob store, all partition files and their index entries
        # of this job go in ONE request
        host = utils.get_hostname()
        outputs, index = [], []
        for p in range(nparts):
            if cols["bounds"][p + 1] == cols["bounds"][p]:
                continue
            s = dev.partition_slice(cols, p)
            name = f"{self.path}/{self.results_ns}.P{p}.M{map_key}"
            outputs.append((name, codec.encode_columnar(s["hi"], s["lo"], s["val"], s["key_off"], s["key_blob"])))
            index.append((INDEX_PREFIX + name + INDEX_SEP + host, b""))
            _dump("map", name, outputs[-1][1])
        self._store_outputs(outputs, index)
        elapsed = _time.process_time() - clock1
        self.mark_as_written(elapsed)
        return elapsed

    # -- reduce --------------------------------------------------------------------
    def _prepare_reduce(self):
        g = modules.field(self.module, "reducefn")
        aci = all(bool(modules.field(self.module, f)) for f in
                  ("associative_reducer", "commutative_reducer", "idempotent_reducer"))
        dev_op = modules.field(self.module, "device_reduce")
        dev_reducefn = modules.field(self.module, "device_reducefn") if dev_op is None else None
        part_key, value = self.get_pair()

        def run():
            clock1 = _time.process_time()
            job_file, res_file, mappers = value["file"], value["result"], value.get("mappers", [])
            fs, _, make_lines_iterator = fsmod.router(self.cnn, mappers, self.storage, self.path)
            import re
            match = {"filename": {"$regex": "^" + re.escape(job_file) + r"\..*"}}
            if self.storage in ("gridfs", "hbm"):
                filenames = [v["filename"] for v in fs.list(match, prefix=job_file + ".")]
            else:
                filenames = [v["filename"] for v in fs.list(match)]
            rstore, rbuilder = result_store(self.cnn, self.storage, self.path)
            rstore.remove_file(res_file)
            blobs = None
            pulled = None
            cols_op = dev_op is not None and dev_op not in FOLD_OPS and _is_cols(dev_op)
            if (dev_op in FOLD_OPS or cols_op) and filenames:
                if self.storage in ("gridfs", "hbm"):  # all inputs (or descriptors) in one round trip per shard
                    blobs = [b or b"" for b in self.cnn.gridfs().get_many(filenames)]
                else:
                    blobs = [fsmod.read_blob(self.cnn, self.storage, self.path, n) for n in filenames]
                if self.storage == "hbm":
                    from . import hbm_store
                    if not all(hbm_store.is_descriptor(b) for b in blobs):
                        raise RuntimeError("hbm storage: a map file's descriptor is missing")
                    if dev_op in FOLD_OPS and dev.default_device().type == "cuda":
                        pulled = blobs  # the files stay on the device (pulled peer to peer below)
                    else:
                        blobs = hbm_store.store().read_many(blobs)
                magic = codec.MAGIC_COL2 if cols_op else codec.MAGIC_COL
                if pulled is None and not all(b[:4] == magic for b in blobs):
                    blobs = None
            b = rbuilder()
            if blobs is not None:
                with dev.PLANE_LOCK:
                    if pulled is not None:
                        out = _device_reduce_hbm(pulled, dev_op)
                    else:
                        out = _device_reduce_cols(blobs, dev_op) if cols_op else _device_reduce(blobs, dev_op)
                b.append(out)
                if _DUMP is not None and pulled is None:
                    import zlib
                    _dump("redin", res_file, "\n".join(f"{n}\t{len(x)}\t{zlib.crc32(x)}" for n, x in
                                                      zip(filenames, blobs)).encode())
                    _dump("redout", res_file, out)
            else:
                merged = utils.merge_iterator(fs, filenames, make_lines_iterator)
                recs = None
                if dev_reducefn is not None:
                    merged = list(merged)
                    with dev.PLANE_LOCK:
                        recs = _device_reduce_lists(merged, self.module)
                if recs is None:
                    recs = []
                    for k, v in merged:
                        if not aci or len(v) > 1:
                            out = []
                            g(k, v, out.append)
                            v = [tuple_(x) for x in out]
                        recs.append((k, v))
                b.append(codec.encode_records(recs))
            b.build(res_file)
            elapsed = _time.process_time() - clock1
            if not self.mark_as_written(elapsed):
                return elapsed
            gfs = self.cnn.gridfs()
            if self.storage in ("gridfs", "hbm"):
                gfs.remove_many(filenames)
            else:
                for n in filenames:
                    fs.remove_file(n)
            ipre = INDEX_PREFIX + job_file + "."
            gfs.remove_many([f["filename"] for f in gfs.list(None, prefix=ipre)])
            return elapsed
        return run


def _aligned_bases(lens) -> tuple[list[int], int]:
    """Offsets of files laid out back to back at 4 mod 16 (an MRC1 file's
    8-byte columns follow its 20-byte header: they are then aligned)."""
    bases, total = [], 0
    for n in lens:
        off = (total + 15) // 16 * 16 + 4
        bases.append(off)
        total = off + n
    return bases, total


def _decode_files(buf: torch.Tensor, bases: list[int], rows: list[int]):
    """MRC1 files at ``bases`` of one device buffer -> (hi, lo, val, rep)
    columns, ONE launch (csrc/hip/ipc.hip); rep words index ``buf``."""
    from ..ops import _hip
    d = buf.device
    rstart = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(rows, out=rstart[1:])
    n = int(rstart[-1])
    meta = torch.from_numpy(np.concatenate([np.asarray(bases, np.int64), rstart])).to(d)
    cols = torch.empty((4, max(n, 1)), dtype=torch.int64, device=d)
    hi, lo, val, rep = (cols[i, :n] for i in range(4))
    _hip.call("mr_mrc1_decode", _hip.ptr(buf), _hip.ptr(meta), len(rows), n, _hip.ptr(hi), _hip.ptr(lo),
              _hip.ptr(val), _hip.ptr(rep), _hip.stream(d))
    return hi, lo, val, rep


def _reduce_device_cols(hi, lo, val, rep, src, op: str) -> bytes:
    d = hi.device
    tab = _reduce_table(d, op, 2 * hi.numel())
    tab.insert(hi, lo, val, rep, src=src)  # long keys verified against their bytes
    out = dev.finalize_table(tab, src, 1, None, need_keys=True)  # one partition: the job's own
    return codec.encode_columnar(out["hi"], out["lo"], out["val"], out["key_off"], out["key_blob"])


def _device_reduce_hbm(descs: list[bytes], op: str) -> bytes:
    """``hbm`` storage: the partition's files are pulled from the map
    workers' device arenas (peer to peer, one launch) and decoded on the
    device (one launch) — no host copy of the intermediate data."""
    from . import hbm_store
    d = dev.default_device()
    buf, bases, ds = hbm_store.store().pull_device(descs, d)
    hi, lo, val, rep = _decode_files(buf, bases, [x["rows"] for x in ds])
    return _reduce_device_cols(hi, lo, val, rep, buf, op)


def _device_reduce(blobs: list[bytes], op: str) -> bytes:
    """Merge columnar partition files on the device: hash-aggregate all
    (key, value) rows, sort, write one columnar result.  On the GPU the files
    go up as they are (one pinned staging copy, one H2D copy) and are decoded
    there by one launch."""
    d = dev.default_device()
    if d.type == "cuda":
        bases, total = _aligned_bases([len(b) for b in blobs])
        stage = torch.empty(max(total, 16), dtype=torch.uint8, pin_memory=True)
        a = stage.numpy()
        for off, b in zip(bases, blobs):
            a[off:off + len(b)] = np.frombuffer(b, np.uint8)
        buf = stage.to(d, non_blocking=True)
        rows = [int(np.frombuffer(b, np.uint64, 1, 4)[0]) for b in blobs]
        hi, lo, val, rep = _decode_files(buf, bases, rows)
        return _reduce_device_cols(hi, lo, val, rep, buf, op)
    cols = [codec.decode_columnar(b) for b in blobs]
    n = sum(int(c["hi"].size) for c in cols)
    hi = torch.from_numpy(np.concatenate([c["hi"] for c in cols]).view(np.int64)).to(d)
    lo = torch.from_numpy(np.concatenate([c["lo"] for c in cols]).view(np.int64)).to(d)
    val = torch.from_numpy(np.concatenate([c["val"] for c in cols])).to(d)
    # key bytes: concatenate blobs, rep = global offset of each key
    bases = np.cumsum([0] + [int(c["key_blob"].size) for c in cols])[:-1]
    offs = np.concatenate([c["key_off"][:-1] + b for c, b in zip(cols, bases)]).astype(np.uint64)
    lens = np.concatenate([np.diff(c["key_off"]) for c in cols]).astype(np.uint64)
    rep = torch.from_numpy(((offs << np.uint64(24)) | lens).view(np.int64)).to(d)
    src = torch.from_numpy(np.concatenate([c["key_blob"] for c in cols] + [np.zeros(1, np.uint8)])).to(d)
    tab = _reduce_table(d, op, 2 * n)
    tab.insert(hi, lo, val, rep, src=src)  # long keys verified against their bytes
    out = dev.finalize_table(tab, src, 1, None, need_keys=True)  # one partition: the job's own
    return codec.encode_columnar(out["hi"], out["lo"], out["val"], out["key_off"], out["key_blob"])


_RED_TABLES: dict = {}


def _reduce_table(d, op: str, need: int):
    """A worker's reduce hash table, kept across its jobs (reset, regrown when
    a job needs more slots)."""
    key = (str(d), op)
    t = _RED_TABLES.get(key)
    if t is None or t.cap < need:
        t = _RED_TABLES[key] = dev.ops.HashTable(max(1024, need), device=d, op=op)
    else:
        t.reset()
    return t


def _is_cols(op) -> bool:
    from ..ops import agg as A
    return A.is_column_spec(op)


def ops_next_pow2(n: int) -> int:
    return 1 << max(0, (int(n) - 1).bit_length())


def _device_reduce_cols(blobs: list[bytes], spec) -> bytes:
    """Merge ``MRC2`` partition files of a typed fold on the device: the
    partial physical columns of every key are folded again (a mean's sums
    and counts add up) and the output columns written."""
    from ..ops import agg as A
    from ..parallel import generic as G
    phys = A.Physical(A.parse_spec(spec))
    cols = [codec.decode_columns(b) for b in blobs]
    d = dev.default_device()
    n = sum(int(c["hi"].size) for c in cols)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d)  # noqa: E731
    hi = t(np.concatenate([c["hi"] for c in cols]).view(np.int64))
    lo = t(np.concatenate([c["lo"] for c in cols]).view(np.int64))
    bases = np.cumsum([0] + [int(c["key_blob"].size) for c in cols])[:-1]
    offs = np.concatenate([c["key_off"][:-1] + b for c, b in zip(cols, bases)]).astype(np.uint64)
    lens = np.concatenate([np.diff(c["key_off"]) for c in cols]).astype(np.uint64)
    rep = t(((offs << np.uint64(24)) | lens).view(np.int64))
    src = t(np.concatenate([c["key_blob"] for c in cols] + [np.zeros(1, np.uint8)]))
    vals = [t(np.concatenate([c["cols"][j] for c in cols])) for j in range(len(phys.cols))]
    merge = [(dt, op, j) for j, (dt, op, _i) in enumerate(phys.cols)]
    cap = max(1024, 4 * n)
    while True:
        tab = A.AggTable(cap, d, merge)
        tab.src = src
        tab.insert(n, vals, hi=hi, lo=lo, rep=rep)
        m, ovf = tab.stats()
        if not ovf:
            break
        cap *= 4
    out = G.order_fold(*tab.compact((m, False)), src, 1, None, phys)
    part = G.host_partitions(out, 1).get(0)
    if part is None:
        return codec.encode_columns(np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                                    [np.zeros(0, c.dtype) for c in G._np_cols(out)], np.zeros(1, np.int64),
                                    np.zeros(0, np.uint8))
    return codec.encode_columns(part["hi"], part["lo"], part["cols"], part["key_off"], part["key_blob"])


def _device_reduce_lists(merged: list, rmod) -> list | None:
    """A reduce job's merged (key, values) lists through the module's
    batched ``device_reducefn`` (parallel/reducers.py) — None when a value
    is not a number (the per-key host reducefn then runs)."""
    from ..parallel import reducers as RD
    from ..parallel.generic import host_partitions
    if not merged:
        return []
    flat = [x for _, v in merged for x in v]
    if not all(isinstance(x, (int, float)) and not isinstance(x, bool) for x in flat):
        return None
    isf = any(isinstance(x, float) for x in flat)
    dtype = "f64" if isf else "i64"
    d = dev.default_device()
    lens = np.array([len(v) for _, v in merged], np.int64)
    off = np.zeros(lens.size + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    val = torch.from_numpy(np.asarray(flat, np.float64 if isf else np.int64)).to(d)
    kb = [k.encode("utf-8", "surrogateescape") if isinstance(k, str) else str(k).encode() for k, _ in merged]
    koff = np.zeros(len(kb) + 1, np.int64)
    np.cumsum([len(k) for k in kb], out=koff[1:])
    blob = np.frombuffer(b"".join(kb), np.uint8) if koff[-1] else np.zeros(0, np.uint8)
    keys = RD.KeyBatch(torch.zeros(len(kb), dtype=torch.int64, device=d),
                       torch.zeros(len(kb), dtype=torch.int64, device=d),
                       key_off=torch.from_numpy(koff).to(d), key_blob=torch.from_numpy(blob.copy()).to(d))
    red = RD.ListReducers(rmod, dtype)
    bits = val.view(torch.int64) if isf else val
    out = red.reduce_device(keys, torch.from_numpy(off).to(d), bits)
    out.update(hi=keys.hi, lo=keys.lo, key_off=keys.key_off, key_blob=keys.key_blob, exact=True,
               counts=torch.tensor([len(kb)], dtype=torch.int64))
    part = host_partitions(out, 1, dtype).get(0)
    ks = [k for k, _ in merged]
    return [(k, list(v)) for k, (_kk, v) in zip(ks, codec.iter_columnar(part))]


def result_store(cnn, storage: str, path: str):
    """Where reduce results live: the coordinator blob store, whatever the
    storage of the intermediate files (results always go to GridFS in the
    reference, job.lua:249-251)."""
    g = cnn.gridfs()
    return g, (lambda: cnn.grid_file_builder())


def utest() -> None:
    f = cached(lambda i: i)
    for _ in range(2):
        for i in range(1, 11):
            assert f(i) == i
