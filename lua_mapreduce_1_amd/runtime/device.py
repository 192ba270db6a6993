"""Device (HBM) data plane of a map/reduce job.

A map module opts in by defining ``device_mapfn(key, value, emit)``; ``emit``
is a :class:`DeviceEmitter` whose calls feed HBM-resident kernels instead of
Python dicts:

* ``emit.words(text_u8)`` — every whitespace token of a byte tensor with value
  1, through the fused tokenize + exact-key + LDS-combine kernel (K1-K5);
* ``emit.spans(starts, lens, vals=None, text=None)`` — keys = byte spans of
  the staged chunk (or ``text``), e.g. CSV fields or n-grams picked with
  ops/text.py and torch ops;
* ``emit.pairs(hi, lo, vals, rep=None, src=None)`` — a batch of (key, value)
  pairs already encoded as 128-bit keys (ops.keys);
* ``emit(key, value)`` — one host pair (buffered, inserted in one batch).

Values are int64 and are folded at insert time with the reduce module's
``device_reduce`` op (``"sum" | "min" | "max" | "count"``), i.e. the combiner of
job.lua:92-96,198-202 runs inside the hash table.  Partitioning uses the
partition module's ``device_partition = ("fnv1", N)`` (exact FNV-1 of the key
bytes mod N, examples/WordCount/partitionfn.lua) or, failing that, the host
``partitionfn`` once per distinct key.
"""
from __future__ import annotations

import atexit
import numpy as np
import torch

from .. import ops
from ..ops import keys as K


_HAS_GPU: bool | None = None
# device map jobs run per device type (observability; tests check that the
# worker's device plane really ran on the GPU)
STATS: dict[str, int] = {}
# finalize() results alias process-wide pinned buffers (_POOL) and the sort /
# tail workspaces are per device: threads of one process that run device jobs
# (several workers in one process) hold this lock around a job
import threading as _threading  # noqa: E402
PLANE_LOCK = _threading.RLock()


def default_device():
    global _HAS_GPU
    if _HAS_GPU is None:  # torch.cuda.is_available() costs ~2.6 ms a call
        _HAS_GPU = torch.cuda.is_available()
    if _HAS_GPU:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


_CTX_CACHE: dict = {}


def warm_worker(op: str = "sum", capacity: int = 1 << 20) -> None:
    """Bring up a worker's GPU device plane before its first job: the HIP
    context and kernel library, the map context (table + arena) that
    :meth:`DeviceMapContext.for_job` hands out, the reduce table, the sort
    and tail workspaces and the pinned download buffers (a tiny map + tail).
    A no-op without a GPU."""
    d = default_device()
    if d.type != "cuda":
        return
    from ..ops import _hip
    from . import job as job_mod
    with PLANE_LOCK:  # (worker threads of one process share the plane's buffers)
        _hip.lib()
        ctx = DeviceMapContext.for_job(op, capacity, d)
        ctx.emit.words(torch.frombuffer(bytearray(b"warm up the device plane\n"), dtype=torch.uint8).to(d))
        finalize_table(ctx.table, ctx.source(), 1, None, need_keys=True)
        STATS["maps_cuda"] = max(0, STATS.get("maps_cuda", 0) - 1)  # (not a job)
        job_mod._reduce_table(d, op, 1 << 21)
        torch.cuda.synchronize(d)


class DeviceMapContext:
    """State of one device map job: the hash table and ONE contiguous device
    byte arena holding every key-byte source the job emitted from (input
    texts, host-pair blobs, emitted key blobs).  Every rep word of the table
    indexes that arena, so long keys are verified byte for byte on insert
    (exact identity) and their bytes are materialised from it at the end."""

    def __init__(self, device=None, op: str = "sum", capacity: int = 1 << 20):
        self.device = torch.device(device) if device is not None else default_device()
        STATS["maps_" + self.device.type] = STATS.get("maps_" + self.device.type, 0) + 1
        self.op = op
        self.capacity = capacity
        self.table = ops.HashTable(capacity, device=self.device, op=op)
        self.arena: torch.Tensor | None = None
        self.sources: list[torch.Tensor] = []  # (engine-owned arenas only: see SPMDEngine._run_map)
        self.base = 0
        self.host_pairs: list[tuple[bytes, int]] = []
        self.emit = DeviceEmitter(self)

    @classmethod
    def for_job(cls, op: str = "sum", capacity: int = 1 << 20, device=None) -> "DeviceMapContext":
        """A worker's device map context, kept across its jobs: the HBM table
        (reset, one kernel) and the byte arena are reused instead of being
        allocated and cleared per job.  Callers hold PLANE_LOCK."""
        d = torch.device(device) if device is not None else default_device()
        key = (str(d), op, int(capacity))
        ctx = _CTX_CACHE.get(key)
        if ctx is None:
            if len(_CTX_CACHE) >= 4:
                _CTX_CACHE.clear()
            ctx = _CTX_CACHE[key] = cls(d, op, capacity)
        else:
            STATS["maps_" + d.type] = STATS.get("maps_" + d.type, 0) + 1
            ctx.table.reset()
            ctx.base = 0
            ctx.sources = []
            ctx.host_pairs = []
            ctx.table.src = ctx.arena
        return ctx

    def add_source(self, t: torch.Tensor) -> tuple[int, torch.Tensor]:
        """Append ``t``'s bytes to the arena; returns (offset, arena view of
        them).  The arena grows by doubling (offsets stay valid)."""
        if self.sources is None:
            raise RuntimeError("a map over engine-staged splits (device_input='split') emits keys whose bytes are "
                               "in its input: words(), or pairs() with rep words relative to the mapped data")
        n = t.numel()
        need = self.base + n
        if self.arena is None or self.arena.numel() < need:
            grown = torch.empty(max(need, 2 * (self.arena.numel() if self.arena is not None else 0), 1 << 16),
                                dtype=torch.uint8, device=self.device)
            if self.arena is not None and self.base:
                grown[:self.base].copy_(self.arena[:self.base])
            self.arena = grown
        b = self.base
        view = self.arena[b:need]
        if n:
            view.copy_(t.reshape(-1), non_blocking=True)
        self.base = need
        self.table.src = self.arena
        return b, view

    def source(self) -> torch.Tensor | None:
        if self.arena is None:
            return None
        return self.arena[:self.base]

    def flush_host_pairs(self) -> None:
        if not self.host_pairs:
            return
        blob = b"".join(k for k, _ in self.host_pairs)
        base, _ = self.add_source(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
        his, los, reps, off = [], [], [], 0
        for k, _ in self.host_pairs:
            h, l_ = K.pack_key(k)
            his.append(h)
            los.append(l_)
            reps.append(K.make_rep(base + off, len(k)))
            off += len(k)
        t = lambda a: torch.from_numpy(np.array(a, dtype=np.uint64).view(np.int64)).to(self.device)  # noqa: E731
        vals = torch.tensor([v for _, v in self.host_pairs], dtype=torch.int64, device=self.device)
        self.table.insert(t(his), t(los), vals, t(reps), src=self.arena)
        self.host_pairs = []

    def grow_and_retry(self, fn) -> None:
        """Run fn(table); on hash-table overflow double the capacity and re-run
        everything (the overflow flag makes the result unusable)."""
        fn(self.table)


class DeviceEmitter:
    def __init__(self, ctx: DeviceMapContext):
        self.ctx = ctx

    @property
    def device(self):
        return self.ctx.device

    def words(self, text: torch.Tensor) -> None:
        """Every whitespace token of ``text`` with value 1 (fused kernel)."""
        ctx = self.ctx
        if ctx.arena is not None and ctx.sources is None:
            # engine-owned arena (SPMDEngine._run_map): ``text`` already lives
            # in it at byte ctx.base
            ctx.table.wordcount_map(text, rep_base=ctx.base, src=ctx.arena)
            ctx.base += text.numel()
            return
        base, view = ctx.add_source(text)
        ctx.table.wordcount_map(view, rep_base=base, src=ctx.arena)

    def spans(self, starts, lens, vals=None, text: torch.Tensor | None = None) -> None:
        """Keys = the byte spans ``text[starts[i] : starts[i] + lens[i]]``
        (default ``text``: the chunk being mapped; empty spans skipped) with
        values ``vals`` (int64 tensor or number; ignored by ``count``)."""
        ctx = self.ctx
        t = text if text is not None else getattr(ctx, "chunk", None)
        if t is None:
            raise ValueError("emit.spans: no staged chunk, pass text=")
        if t.device != ctx.device:
            t = t.to(ctx.device)
        if ctx.op == "count":
            vals = None
        if ctx.arena is not None and ctx.sources is None:
            # engine-owned arena: the spans must lie in the staged input
            base = t.data_ptr() - ctx.arena.data_ptr()
            if not (0 <= base and base + t.numel() <= ctx.arena.numel()):
                raise ValueError("emit.spans: with staged splits, text must be a view of the staged input")
        else:
            base, t = ctx.add_source(t)
        ctx.table.insert_spans(t, starts, lens, vals, rep_base=base, src=ctx.arena)

    def pairs(self, hi, lo, vals=None, rep=None, src: torch.Tensor | None = None) -> None:
        """A batch of encoded (key, value) pairs; long keys' rep words index
        ``src`` (appended to the job's arena)."""
        ctx = self.ctx
        if ctx.op == "count":
            vals = None
        add = 0
        if src is not None:
            add, _ = ctx.add_source(src)
        elif ctx.sources is None:
            add = ctx.base  # engine-staged input: rep words relative to the mapped data
        ctx.table.insert(hi, lo, vals, rep, rep_add=add, src=ctx.arena)

    def error_word(self):
        """The current map chunk's device error word (int32[1] on the
        device; None off the SPMD engine / on CPU): device code that finds the
        chunk's input bad writes it non-zero, and the engine re-runs the
        chunk's jobs (BROKEN) or drops them (FAILED after MAX_JOB_RETRIES)."""
        return getattr(self.ctx, "err_word", None)

    def __call__(self, key, value=1) -> None:
        if isinstance(key, str):
            key = key.encode("utf-8", "surrogateescape")
        elif not isinstance(key, bytes):
            key = str(key).encode()
        self.ctx.host_pairs.append((key, 1 if self.ctx.op == "count" else int(value)))


# ---------------------------------------------------------------------------
def partition_of(hi, lo, rep, src, nparts: int, partition_module=None) -> torch.Tensor:
    spec = getattr(partition_module, "device_partition", None) if partition_module is not None else None
    if spec is None and partition_module is None:
        spec = ("fnv1", nparts)
    if spec is not None:
        kind, n = spec
        if kind != "fnv1":
            raise ValueError(f"unknown device partition {kind}")
        part, _ = ops.key_meta(hi, lo, rep, src, nparts=n, want_len=False)
        return part
    # host partitionfn once per distinct key
    f = getattr(partition_module, "partitionfn")
    kb = ops.key_bytes_list(hi.cpu(), lo.cpu(), rep.cpu(), src.cpu() if src is not None else None)
    p = [int(f(k.decode("utf-8", "surrogateescape"))) for k in kb]
    return torch.tensor(p, dtype=torch.int32, device=hi.device)


def fix_long_key_order(hi: np.ndarray, lo: np.ndarray, off: np.ndarray, blob: np.ndarray):
    """Permutation that makes key order exactly bytewise.

    Keys are sorted by (hi, lo); for long keys lo is a hash, so runs sharing the
    8-byte prefix ``hi`` that contain a long key are re-sorted by their bytes.
    Returns None when the order is already exact (the common case).
    """
    n = hi.size
    if n < 2:
        return None
    is_long = (lo & np.uint64(0xFF)) == np.uint64(0xFF)
    if not is_long.any():
        return None
    same = hi[1:] == hi[:-1]
    if not ((is_long[1:] | is_long[:-1]) & same).any():
        return None
    perm = np.arange(n)
    starts = np.flatnonzero(np.concatenate([[True], ~same]))
    ends = np.concatenate([starts[1:], [n]])
    has_long = np.add.reduceat(is_long.astype(np.int64), starts) > 0
    b = blob.tobytes() if isinstance(blob, np.ndarray) else bytes(blob)
    changed = False
    for s, e in zip(starts[has_long], ends[has_long]):
        if e - s > 1:
            idx = list(range(s, e))
            idx.sort(key=lambda i: b[off[i]:off[i + 1]])
            if idx != list(range(s, e)):
                perm[s:e] = idx
                changed = True
    return perm if changed else None


class _PinnedPool:
    """Reusable pinned host buffers for device -> host result copies.
    ``gen`` counts the downloads into them (finalize_host): a result whose
    columns alias the pool is stale once ``gen`` has moved on."""

    def __init__(self):
        self.bufs: dict[str, torch.Tensor] = {}
        self.gen = 0

    def get(self, name: str, n: int, dtype) -> torch.Tensor:
        b = self.bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            if b is not None:
                wait_downloads()  # a download in flight may still write the buffer being replaced
            b = torch.empty(max(n, 1024) * 5 // 4, dtype=dtype, pin_memory=default_device().type == "cuda")
            self.bufs[name] = b
        return b[:n]


_POOL = _PinnedPool()
_BLOB_EST: dict = {}  # device -> expected key-blob bytes of the next finalize()


_SDMA: dict = {}  # device -> [(dst, src, nbytes)] downloads deferred to flush_downloads
_INFLIGHT: dict = {}  # device -> the Downloads batch still landing (flush_downloads(wait=False))


def _sdma_ok() -> bool:
    ok = _SDMA.get("ok")
    if ok is None:
        from ..ops import _hip
        ok = _SDMA["ok"] = bool(_hip.lib().mr_sdma_available())
    return ok


def dma_to_host(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Queue a device -> pinned-host download of ``src`` into ``dst`` on the
    current stream (hipMemcpyAsync; not torch's non_blocking copy_, which
    also records an event for the pinned block in its host allocator on
    every call — that event pool's growth stalled the host for ~5 ms now and
    then).  A download of at least ``MR_SDMA_MIN_MB`` is deferred instead: the
    runtime would run it as a blit kernel on the CUs, beside the next
    iteration's map; :func:`flush_downloads` (after the stream wait that
    precedes every read of the results) moves it on the SDMA engines."""
    from ..ops import _hip
    from ..utils.config import TUNABLES
    assert src.is_contiguous() and dst.is_contiguous() and dst.numel() * dst.element_size() >= \
        src.numel() * src.element_size()
    nb = src.numel() * src.element_size()
    if TUNABLES.sdma_min_mb > 0 and nb >= TUNABLES.sdma_min_mb * (1 << 20) and _sdma_ok():
        _SDMA.setdefault(src.device, []).append((dst, src, nb))
        return
    b = _INFLIGHT.get(src.device)
    if b is not None and b.writes(dst.data_ptr(), nb):
        b.wait()  # a lazy batch still fills this buffer: it must not land over this copy
    _hip.call("mr_d2h_async", _hip.ptr(dst), _hip.ptr(src), nb, _hip.stream(src.device))


class Downloads:
    """A batch of SDMA downloads still landing in pinned host memory
    (``flush_downloads(wait=False)``).  It holds the device sources, so their
    memory is not reused before the copies are done; :meth:`wait` blocks until
    the bytes are in place (and redoes the copies through hipMemcpy if the
    engine reported an error)."""

    def __init__(self, device, handle: int, pend: list):
        self.device, self.handle, self.pend = device, handle, pend

    @property
    def done(self) -> bool:
        return self.pend is None

    def writes(self, ptr: int, nbytes: int) -> bool:
        """True if a copy of this batch (still in flight) writes into [ptr, ptr + nbytes)."""
        return any(d.data_ptr() < ptr + nbytes and ptr < d.data_ptr() + nb for d, _s, nb in (self.pend or ()))

    def wait(self) -> None:
        if self.pend is None:
            return
        from ..ops import _hip
        pend, self.pend = self.pend, None
        if _INFLIGHT.get(self.device) is self:
            del _INFLIGHT[self.device]
        if _hip.lib().mr_sdma_wait(self.handle) < 0:
            _SDMA["ok"] = False
            for dst, src, nb in pend:  # blocking runtime copies
                dst.view(torch.uint8)[:nb].copy_(src.view(torch.uint8)[:nb])


def wait_downloads(device=None) -> None:
    """Wait for the in-flight download batch of ``device`` (None: of every
    device) — before anything rewrites or frees the pinned buffers it fills."""
    for d in ([device] if device is not None else list(_INFLIGHT)):
        b = _INFLIGHT.get(d)
        if b is not None:
            b.wait()


atexit.register(wait_downloads)  # no copy may still read device memory the process is freeing


def discard_downloads(device) -> None:
    """Drop the downloads deferred for a tail whose results are thrown away."""
    _SDMA.pop(device, None)


def flush_downloads(device, wait: bool = True):
    """Run the downloads deferred by :func:`dma_to_host` on the SDMA engines
    (call after waiting for the stream that produced them).  ``wait=True``:
    return once they landed.  ``wait=False``: return a :class:`Downloads`
    batch still in flight (None when nothing is left to wait for); the caller
    waits on it before reading the buffers.  A batch still landing from an
    earlier call is waited for first (the pinned buffers are shared)."""
    wait_downloads(device)
    pend = _SDMA.pop(device, None)
    if not pend:
        return None
    import ctypes
    from ..ops import _hip
    n = len(pend)
    dsts = (ctypes.c_void_p * n)(*[t[0].data_ptr() for t in pend])
    srcs = (ctypes.c_void_p * n)(*[t[1].data_ptr() for t in pend])
    sizes = (ctypes.c_uint64 * n)(*[t[2] for t in pend])
    if wait:
        rc = _hip.lib().mr_sdma_d2h(dsts, srcs, sizes, n)
        if rc < 0:
            raise RuntimeError("device -> host download failed (SDMA and hipMemcpy)")
        if rc == 1:
            _SDMA["ok"] = False  # the SDMA path failed once: plain runtime copies from now on
        return None
    fell = ctypes.c_int(0)
    h = int(_hip.lib().mr_sdma_d2h_begin(dsts, srcs, sizes, n, ctypes.byref(fell)))
    if h == (1 << 64) - 1:
        raise RuntimeError("device -> host download failed (SDMA and hipMemcpy)")
    if fell.value:
        _SDMA["ok"] = False
    if h == 0:
        return None
    b = _INFLIGHT[device] = Downloads(device, h, pend)
    return b


def _to_host(t: torch.Tensor, name: str) -> torch.Tensor:
    if not t.is_cuda:
        return t
    h = _POOL.get(name, t.numel(), t.dtype)
    dma_to_host(h, t.contiguous())
    return h


def finalize(hi, lo, val, rep, src, nparts: int, partition_module=None, part: torch.Tensor | None = None,
             _presorted: bool = False, need_keys: bool = False, _exact: bool = False, blob_cap: int | None = None):
    """Partition, sort by (partition, key) and materialise key bytes.

    Returns a dict of host numpy arrays: hi, lo, val, key_off, key_blob and
    ``bounds`` (partition p occupies rows bounds[p]:bounds[p+1]).  All device
    work is queued first; results come back through reusable pinned buffers
    with a single synchronisation.  NOTE: the arrays alias the pinned pool and
    stay valid until the next finalize() call (copy them to keep them longer).
    """
    pend = finalize_device(hi, lo, val, rep, src, nparts, partition_module, part, _presorted, blob_cap=blob_cap)
    pend["exact"] = _exact
    try:
        return finalize_host(pend, partition_module, need_keys)
    except BlobCapacityError as e:  # keys overlapping in their source (n-gram spans)
        pend = finalize_device(hi, lo, val, rep, src, nparts, partition_module, part, _presorted, blob_cap=e.nbytes)
        return finalize_host(pend, partition_module, need_keys)


class TailBoundError(RuntimeError):
    """A padded tail (finalize_table_native(padded=True)) was launched for
    fewer rows than its table holds, or its table overflowed: re-run it with
    the table's count (``overflow``: grow and refill the table first)."""

    def __init__(self, overflow: bool):
        super().__init__("reduce table overflowed" if overflow else "reduce tail row bound too small")
        self.overflow = overflow


class BlobCapacityError(RuntimeError):
    """The key bytes of a result exceed the blob capacity the tail was given
    (keys that overlap in their source, e.g. n-gram spans, can need more
    bytes than the source holds): re-run the tail with ``blob_cap=nbytes``."""

    def __init__(self, nbytes: int, cap: int):
        super().__init__(f"key bytes ({nbytes}) exceed the blob capacity ({cap})")
        self.nbytes = nbytes


def finalize_device(hi, lo, val, rep, src, nparts: int, partition_module=None, part: torch.Tensor | None = None,
                    _presorted: bool = False, blob_cap: int | None = None,
                    lengths: torch.Tensor | None = None, counts: torch.Tensor | None = None) -> dict:
    """The device half of :func:`finalize`: every kernel and device->pinned
    copy, no host synchronisation (so it can be captured in a hipGraph once
    the pinned buffers exist).  Returns the pending state for finalize_host.
    ``counts`` (presorted rows): the rows per partition when the caller has
    them (int64 [nparts] on the device)."""
    n = hi.numel()
    if part is None:
        part = partition_of(hi, lo, rep, src, nparts, partition_module)
    args = (hi, lo, val, rep)
    if _presorted:
        bad = torch.zeros(1, dtype=torch.int32, device=hi.device)
    else:
        part, hi, lo, val, rep, bad = ops.sort_by_partition_key(part, hi, lo, val, rep, nparts,
                                                                src=src if hi.is_cuda else None)
    pend = {"n": n, "nparts": nparts, "args": args, "src": src, "presorted": _presorted, "hi": hi, "lo": lo}
    if not hi.is_cuda:
        off, blob = ops.gather_key_bytes(hi, lo, rep, src)
        counts = ops.bincount(part, nparts) if n else torch.zeros(nparts, dtype=torch.int64)
        pend.update(val=val, off=off, blob=blob, counts=counts)
        return pend
    # blob capacity bound: distinct words occupy disjoint bytes of their
    # source (a caller whose keys overlap there passes blob_cap)
    cap = max(src.numel() if src is not None else max(16 * n, 1), blob_cap or 0)
    off, blob = ops.gather_key_bytes(hi, lo, rep, src, lengths=lengths if _presorted else None, capacity=cap)
    if counts is None or not _presorted:
        counts = ops.bincount(part, nparts) if n else torch.zeros(nparts, dtype=torch.int64, device=hi.device)
    hv = _to_host(val, "val")
    ho = _to_host(off.to(torch.int32), "off32") if cap < 2**31 else _to_host(off, "off64")
    est = _BLOB_EST.get(hi.device)
    if est is not None:
        # steady state: DMA (SDMA engine, full PCIe rate) a little more than
        # last time's size; the rare overflow is topped up after the sync
        est = min(est, blob.numel())
        hb = _POOL.get("blob", max(est, 1 << 16), torch.uint8)
        dma_to_host(hb[:est], blob[:est])
    else:
        hb = _POOL.get("blob", max(1 << 20, 16 * n), torch.uint8)
        wait_downloads(hi.device)  # (a lazy batch may still fill hb)
        ops.copy_to_host(blob, hb, off[n:])  # size read on the device: no sync before the copy
    pend.update(off=off, blob=blob, est=est, hv=hv, ho=ho, hb=hb, hc=_to_host(counts, "counts"),
                hbad=_to_host(bad, "bad"), hnb=_to_host(off[n:n + 1], "offn"))  # the key-byte total
    return pend


_TAIL_WS: dict = {}  # device -> (workspace uint8 tensor, {layout key: (offsets, views)})
_TB = {name: i for i, name in enumerate(
    "HI0 LO0 VAL0 REP0 C PART0 ZERO K0 K1 P0 P1 HI LO VAL REP PART LN OFF PARTIALS BLOB PACKED BHIST".split())}
_TAIL_GRAN: dict = {}  # device -> the tail sort's look-back granules (a buffer of their own: mr_tail_run)


def _tail_gran(d, n: int) -> torch.Tensor:
    """Look-back granules of the fused tail's sort: zeroed when allocated and
    never holding anything else, so a granule slot a pass reads before its
    predecessor published is either zero or an older pass's epoch-tagged
    entry — never a stale data word whose bits look like a live tag."""
    from ..ops import _hip
    need = 256 * int(_hip.lib().mr_onesweep_tiles(max(n, 1)))
    g = _TAIL_GRAN.get(d)
    if g is None or g.numel() < need:
        g = _TAIL_GRAN[d] = torch.zeros(max(need, 256 * 64), dtype=torch.int64, device=d)
    return g


def _tail_ws(d, n: int, nparts: int, blob_cap: int, cap: int):
    """Workspace of mr_tail_run (csrc/hip/tail.hip) for a table of ``cap``
    slots and int64 views of the buffers the host half reads, cached per (n,
    nparts, blob capacity, table capacity)."""
    import ctypes
    from ..ops import _hip
    lib = _hip.lib()
    offs = (ctypes.c_uint64 * len(_TB))()
    need = int(lib.mr_tail_ws_layout(ctypes.c_uint64(n), ctypes.c_uint32(nparts), ctypes.c_uint64(blob_cap),
                                     ctypes.c_uint64(cap), offs))
    ws, views = _TAIL_WS.get(d, (None, {}))
    if ws is None or ws.numel() < need:
        ws = torch.zeros(need + need // 4, dtype=torch.uint8, device=d)
        views = {}
    key = (n, nparts, blob_cap, cap)
    v = views.get(key)
    if v is None:
        o = list(offs)
        m = max(n, 1)
        i64 = lambda b, k: ws[o[_TB[b]]:o[_TB[b]] + 8 * k].view(torch.int64)  # noqa: E731
        v = {"args": tuple(i64(b, n) for b in ("HI0", "LO0", "VAL0", "REP0")), "hi": i64("HI", n), "lo": i64("LO", n),
             "off": i64("OFF", m + 1), "blob": ws[o[_TB["BLOB"]]:o[_TB["BLOB"]] + max(blob_cap, 1)],
             # (MR_DEBUG_TAIL: the packed download, the final permutation and sorted keys)
             "packed": ws[o[_TB["PACKED"]]:], "p1": ws[o[_TB["P1"]]:o[_TB["P1"]] + 4 * n],
             "k1": i64("K1", n), "c": i64("C", n), "zero": ws[o[_TB["ZERO"]]:o[_TB["ZERO"]] + 10512]}
        if len(views) > 8:
            views.clear()
        views[key] = v
    _TAIL_WS[d] = (ws, views)
    return ws, v


_CP_WS: dict = {}


def compact_partition(table, n: int, src, nparts: int):
    """Occupied slots of a table -> dense (hi, lo, val, rep) + exact FNV-1
    partition (int32), in ONE kernel (tail_compact; its composite sort key and
    digit histograms are by-products).  The send side of the shuffle; buffers
    are reused across iterations (valid until the next call)."""
    from ..ops import _hip
    d = table.device
    ws = _CP_WS.get(d)
    m = max(n, 1)
    if ws is None or ws["cap"] < m:
        c = m + m // 4
        ws = {"cap": c, "cols": torch.empty((6, c), dtype=torch.int64, device=d),
              "part": torch.empty(c, dtype=torch.int32, device=d),
              "small": torch.empty(1 + 1024 + 256, dtype=torch.int64, device=d)}
        _CP_WS[d] = ws
    nbh = int(_hip.lib().mr_tail_bhist_bytes(table.cap))
    if ws.get("bhist") is None or ws["bhist"].numel() < nbh:
        ws["bhist"] = torch.empty(nbh, dtype=torch.uint8, device=d)
    cols, part, small = ws["cols"], ws["part"], ws["small"]
    hi, lo, val, rep, c = (cols[i, :n] for i in range(5))
    _hip.call("mr_tail_compact", *table._gtab(), table.cap, nparts, _hip.ptr(src), _hip.ptr(hi), _hip.ptr(lo),
              _hip.ptr(val), _hip.ptr(rep), _hip.ptr(part), _hip.ptr(c), _hip.ptr(small[:1]),
              None, None, _hip.ptr(ws["bhist"]), n, n, 0, None, _hip.stream(d))  # no digit histograms here
    return hi, lo, val, rep, part[:n]


def finalize_table_native(table, n: int, src, nparts: int, blob_cap: int | None = None,
                          padded: bool = False) -> dict:
    """Fused device tail straight from an HBM hash table, every launch and
    download queued by ONE native call (mr_tail_run, csrc/hip/tail.hip):
    compact + FNV partition + composite key + digit histograms in one kernel,
    the composite onesweep sort (no histogram pass), one gather that also
    yields key lengths, the exact-order tie fix-up, key bytes, and ONE packed
    download of values/offsets/partition counts (+ the key-byte DMA).  ``n``
    = occupied slots (table.stats()).  Requires nparts <= 256; returns the
    pending state for finalize_host.

    ``padded=True``: ``n`` is a BOUND on the occupied slots (nparts <= 255),
    so nothing is read before the tail is queued: the rows past the count are
    sentinels sorted last, finalize_host takes the count from the partition
    counts, and raises :class:`TailBoundError` if the bound was too small or
    the table overflowed (the caller re-runs with the count)."""
    from ..ops import _hip
    d = table.device
    cap = max(src.numel(), blob_cap or 0)
    ws, v = _tail_ws(d, n, nparts, cap, table.cap)
    nb = int(_hip.lib().mr_tail_pack_bytes(n, nparts))
    hp = _POOL.get("pack", nb, torch.uint8)
    est = _BLOB_EST.get(d)
    if est is not None:
        est = min(est, cap)
        hb = _POOL.get("blob", max(est, 1 << 16), torch.uint8)
        est_arg = est
    else:
        hb = _POOL.get("blob", max(1 << 20, 16 * n), torch.uint8)
        est_arg = -1
    b = _INFLIGHT.get(d)
    if b is not None and (b.writes(hp.data_ptr(), hp.numel()) or b.writes(hb.data_ptr(), hb.numel())):
        b.wait()  # the native tail downloads into these pinned buffers on its stream
    _hip.call("mr_tail_run", *table._gtab(), table.cap, n, nparts, _hip.ptr(src), _hip.ptr(ws),
              _hip.ptr(_tail_gran(d, n)), cap, _hip.ptr(hp), _hip.ptr(hb), est_arg, hb.numel(), 1 if padded else 0,
              _hip.stream(d))
    out = {"n": n, "nparts": nparts, "args": v["args"], "src": src, "presorted": False, "hi": v["hi"], "lo": v["lo"],
           "fused": True, "hp": hp, "off": v["off"], "blob": v["blob"], "est": est, "hb": hb, "padded": padded}
    if _DEBUG_TAIL:
        out.update(dbg_packed=v["packed"][:nb], dbg_perm=v["p1"], dbg_keys=v["k1"], dbg_c=v["c"], dbg_zero=v["zero"])
    return out


# diagnosis: MR_DEBUG_TAIL=1 checks every fused tail after a full device sync:
# the pinned download as the host read it against the device buffer, the
# final sort permutation (a bijection) and the sorted keys' order; a
# difference is reported on stderr as "# DEBUG TAIL"
import os as _os  # noqa: E402
_DEBUG_TAIL = bool(_os.environ.get("MR_DEBUG_TAIL"))


def _debug_tail_check(pend: dict, snap: np.ndarray, blob_snap) -> None:
    import sys
    torch.cuda.synchronize()
    n = pend["n"]
    dev_pack = pend["dbg_packed"].cpu().numpy()
    bad_pack = np.flatnonzero(dev_pack[:snap.size] != snap[:dev_pack.size])
    perm = pend["dbg_perm"].cpu().numpy().view(np.uint32)[:n] if n else np.zeros(0, np.uint32)
    perm_ok = bool(n == 0 or (int(perm.max()) < n and np.bincount(perm, minlength=n).max() == 1))
    keys = pend["dbg_keys"].cpu().numpy().view(np.uint64)[:n]
    order_ok = bool(n < 2 or (keys[1:] >= keys[:-1]).all())
    bad_blob = 0
    if blob_snap is not None and blob_snap.size:
        dev_blob = pend["blob"][:blob_snap.size].cpu().numpy()
        bad_blob = int((dev_blob != blob_snap).sum())
    if bad_pack.size or not perm_ok or not order_ok or bad_blob:
        sys.stderr.write(f"# DEBUG TAIL: n={n} pack bytes {dev_pack.size}: {bad_pack.size} stale (first "
                         f"{bad_pack[:4].tolist()}), perm ok {perm_ok}, order ok {order_ok}, stale blob bytes "
                         f"{bad_blob}\n")
        # the sort's inputs and control words: the composite keys (unchanged by
        # the sort), their digit histograms as the compaction counted them,
        # the per-pass tile counters and the error word
        c = pend["dbg_c"].cpu().numpy().view(np.uint64)[:n]
        z = pend["dbg_zero"].cpu().numpy()
        gh = z[8:8 + 8192].view(np.uint32).reshape(8, 256)
        want = np.stack([np.bincount(((c >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.int64), minlength=256)
                         for b in range(8)]).astype(np.uint32)
        tiles = z[10248:10248 + 32].view(np.uint32)
        err, badw = z[10504:10508].view(np.uint32)[0], z[10508:10512].view(np.uint32)[0]
        ref = np.sort(c)
        wrong = np.flatnonzero(ref != keys)
        from ..ops import _hip
        sys.stderr.write(f"#   ghist ok {bool((gh == want).all())} (bad digits {np.flatnonzero((gh != want).any(1)).tolist()}),"
                         f" tile counters {tiles.tolist()} (tiles {int(_hip.lib().mr_onesweep_tiles(n))}), err {err}, "
                         f"bad {badw}, keys out of place {wrong.size} first {wrong[:3].tolist()} last "
                         f"{wrong[-3:].tolist()}, distinct keys {np.unique(c).size}\n")
        sys.stderr.flush()


def finalize_exact_device(hi, lo, val, rep, src, nparts: int, partition_module=None,
                          blob_cap: int | None = None, aos: torch.Tensor | None = None) -> dict:
    """The device half of a tail ordered exactly by key bytes from the start
    (ops.exact_key_perm) — for key sets whose fused tail falls back every time.
    Keys past the exact sort's length limit get the (partition, hi, lo) sort
    and the host fix-up instead.  Partitions and key lengths come from one
    key_meta pass (device FNV-1 partitions); the rows and their lengths are
    reordered by one gather launch (from the 32-byte row records ``aos`` of
    the compaction when given: one record read per row instead of one line
    per column)."""
    spec = getattr(partition_module, "device_partition", None) if partition_module is not None else ("fnv1", nparts)
    klen = w1 = k7 = None
    if hi.is_cuda and spec is not None and spec[0] == "fnv1" and int(spec[1]) == nparts:
        # partitions, lengths, key bytes 8..15 and the 7-bit sort words in one pass over the key bytes
        if src is not None:
            part, klen, w1, k7 = ops.key_meta(hi, lo, rep, src, nparts=nparts, want_w1=True, want_k7=True)
        else:
            part, klen = ops.key_meta(hi, lo, rep, src, nparts=nparts)
    else:
        part = partition_of(hi, lo, rep, src, nparts, partition_module)
    got = ops.exact_key_perm(part, hi, lo, rep, src, nparts, klen=klen, with_part=True,
                             with_counts=hi.is_cuda, w1=w1, k7=k7, perm32=True) if src is not None else None
    exact = got is not None
    spart = counts = None
    if got is None:
        perm = ops.sort_keys_checked([part.to(torch.int64), hi, lo],
                                     bits=[max(8, int(nparts - 1).bit_length()), 64, 64]).long()
    elif hi.is_cuda:
        perm, spart, counts = got
    else:
        perm, spart = got
    if hi.is_cuda and spart is not None:
        # one gather launch for the four key/value columns; the partitions
        # come sorted from the sort and the lengths from (lo, rep) of the
        # gathered rows (no key bytes read)
        from ..ops import _hip
        n = hi.numel()
        if aos is not None:
            *cols, slen = ops.gather_aos4(perm, aos, want_len=True)
        else:
            cols = [torch.empty(n, dtype=torch.int64, device=hi.device) for _ in range(4)]
            _hip.call("mr_gather_cols", _hip.ptr(perm.to(torch.int32)), n, _hip.ptr(hi), _hip.ptr(lo),
                      _hip.ptr(val), _hip.ptr(rep), None, None, *[_hip.ptr(c) for c in cols], None, None,
                      _hip.stream(hi.device))
            _, slen = ops.key_meta(cols[0], cols[1], cols[3], src, want_part=False)
        pend = finalize_device(*cols, src, nparts, partition_module, part=spart.to(torch.int32), _presorted=True,
                               blob_cap=blob_cap, lengths=slen, counts=counts)
    else:
        pend = finalize_device(hi[perm], lo[perm], val[perm], rep[perm], src, nparts, partition_module,
                               part=part[perm], _presorted=True, blob_cap=blob_cap)
    pend["exact"] = exact
    return pend


def finalize_table(table, src, nparts: int, partition_module=None, need_keys: bool = False) -> dict:
    """HBM table -> host result columns (a worker's map tail): the fused
    native tail (one call: compact, FNV partition, sort, key bytes, one
    download) when the partition is the device FNV-1 of ``nparts`` <= 256
    partitions, else compaction + :func:`finalize`.  An overflowed table
    raises OverflowError."""
    n, ovf = table.stats()
    if ovf:
        raise OverflowError("device map table overflow")
    spec = getattr(partition_module, "device_partition", None) if partition_module is not None else ("fnv1", nparts)
    if (table.is_cuda and src is not None and spec is not None and spec[0] == "fnv1" and int(spec[1]) == nparts
            and 0 < nparts <= 256 and n > 0):
        cap = None
        for _ in range(4):
            try:
                return finalize_host(finalize_table_native(table, n, src, nparts, blob_cap=cap), partition_module,
                                     need_keys)
            except BlobCapacityError as e:
                cap = e.nbytes + e.nbytes // 4 + 4096
    hi, lo, val, rep = table.compact((n, ovf))
    return finalize(hi, lo, val, rep, src, nparts, partition_module, need_keys=need_keys)


def _unpack_fused(pend: dict):
    """(val int64[n], off int32[n+1], counts int64[nparts], bad) views of the packed download."""
    n, nparts = pend["n"], pend["nparts"]
    raw = pend["hp"].numpy()
    offb = ((4 * (n + 1)) + 7) & ~7
    val = raw[:8 * n].view(np.int64)
    off = raw[8 * n:8 * n + 4 * (n + 1)].view(np.int32)
    counts = raw[8 * n + offb:8 * n + offb + 8 * nparts].view(np.int64)
    bad = int(raw[8 * n + offb + 8 * nparts:8 * n + offb + 8 * nparts + 4].view(np.uint32)[0])
    return val, off, counts, bad


def pool_generation() -> int:
    return _POOL.gen


def finalize_host(pend: dict, partition_module=None, need_keys: bool = False, lazy: bool = False) -> dict:
    """The host half of :func:`finalize`: one synchronisation, then numpy.

    ``lazy=True`` (the unfused tail, e.g. the exact key order of n-grams):
    the large downloads (values, key offsets, key bytes) are left landing on
    the SDMA engines and the returned dict carries their
    :class:`Downloads` batch under ``"_downloads"``; its arrays may be read
    only after ``wait()``.  The host can meanwhile queue the next iteration's
    tail, so the GPU does not idle through the transfer.  The counts, the
    flags and the key-byte total are small stream-ordered copies and are read
    here either way, so every error below is still raised eagerly."""
    _POOL.gen += 1
    n, nparts = pend["n"], pend["nparts"]
    hi, lo = pend["hi"], pend["lo"]
    defer = False
    if hi.is_cuda:
        from ..ops import _hip
        _hip.wait_stream(hi.device)
        defer = lazy and not pend.get("fused") and not need_keys and "hnb" in pend
        if not defer:
            flush_downloads(hi.device)  # large downloads: on the SDMA engines, now that their data is produced
        hb, est, blob = pend["hb"], pend["est"], pend["blob"]
        if pend.get("fused") and _DEBUG_TAIL:
            snap = pend["hp"].numpy().copy()  # the download as the host reads it now
            nb0 = int(snap[8 * pend["n"]:8 * pend["n"] + 4 * (pend["n"] + 1)].view(np.int32)[-1]) if pend["n"] else 0
            bsnap = hb.numpy()[:min(nb0, hb.numel(), est if est is not None else nb0)].copy() if nb0 > 0 else None
            _debug_tail_check(pend, snap, bsnap)
        if pend.get("fused"):
            f_val, f_off, f_counts, f_bad = _unpack_fused(pend)
            if pend.get("padded"):
                if f_bad & 24:
                    raise TailBoundError(bool(f_bad & 16))
                # the real rows: their count from the partition counts (the
                # sentinel rows past it sort last and have empty keys)
                n = int(f_counts.sum())
                f_val, f_off = f_val[:n], f_off[:n + 1]
                hi, lo = hi[:n], lo[:n]
                pend = dict(pend, n=n, args=tuple(a[:n] for a in pend["args"]))
            nbytes = int(f_off[n]) if n else 0
        else:
            ho = pend["ho"]
            nbytes = int(pend["hnb"][0]) if n and "hnb" in pend else (int(ho[n]) if n else 0)
        flag = f_bad if pend.get("fused") else int(pend["hbad"][0])
        if defer and (flag & 7 or nbytes > blob.numel() or (est is not None and nbytes > est)
                      or nbytes > hb.numel() or (pend["presorted"] and not pend.get("exact"))):
            # a re-run, a top-up copy or the host fix-up follows: nothing stays in flight
            if flag & 5 or (nbytes > blob.numel() and not flag & 4):
                discard_downloads(hi.device)  # these results are thrown away
            else:
                flush_downloads(hi.device)
            defer = False
        if nbytes > blob.numel() and not flag & 4:
            raise BlobCapacityError(nbytes, blob.numel())
        if nbytes > blob.numel():
            nbytes = blob.numel()  # a given-up sort's rows: discarded below (re-sort)
        if est is not None and nbytes > est:  # grew past the estimate: copy the rest
            hb = _POOL.get("blob", nbytes, torch.uint8)
            hb.copy_(blob[:nbytes])
        elif nbytes > hb.numel():  # kernel path clamped the copy: grow and copy again (rare)
            hb = _POOL.get("blob", nbytes, torch.uint8)
            hb.copy_(blob[:nbytes])
        _BLOB_EST[hi.device] = nbytes + nbytes // 16 + 4096
        hb = hb[:nbytes]
        if flag & 5:
            # bit 0: a tie run was too long for the fixup kernel; bit 2: the
            # radix sort's decoupled look-back gave up (its order is invalid)
            # -> redo with the full multi-word sort, checked (raises if the
            # look-back keeps giving up)
            if flag & 4:
                import sys
                sys.stderr.write("# warning: radix sort look-back gave up; re-sorting\n")
            ahi, alo, aval, arep = pend["args"]
            src = pend["src"]
            p2 = partition_of(ahi, alo, arep, src, nparts, partition_module)
            # exact bytewise order on the device (long keys compared by their
            # bytes); the host fix-up is left for keys past its length limit
            perm = ops.exact_key_perm(p2, ahi, alo, arep, src, nparts) if src is not None else None
            exact = perm is not None
            if perm is None:
                perm = ops.sort_keys_checked([p2.to(torch.int64), ahi, alo],
                                             bits=[max(8, int(nparts - 1).bit_length()), 64, 64]).long()
            out = finalize(ahi[perm], alo[perm], aval[perm], arep[perm], src, nparts, partition_module,
                           part=p2[perm], _presorted=True, need_keys=need_keys, _exact=exact,
                           blob_cap=max(int(blob.numel()), nbytes))
            out["exact_fallback"] = exact
            return out
        # offsets stay int32 when the blob is < 2 GiB (no host-side widening pass)
        if pend.get("fused"):
            h_val, h_off, h_blob, h_counts = f_val, f_off, hb.numpy(), f_counts
        else:
            h_val, h_off, h_blob, h_counts = pend["hv"].numpy(), ho.numpy(), hb.numpy(), pend["hc"].numpy()
        need_fix = bool(flag & 2) or (pend["presorted"] and not pend.get("exact"))
        h_hi = hi.cpu().numpy().view(np.uint64) if (need_fix or need_keys) else None
        h_lo = lo.cpu().numpy().view(np.uint64) if (need_fix or need_keys) else None
    else:
        h_hi, h_lo = hi.numpy().view(np.uint64), lo.numpy().view(np.uint64)
        h_val, h_off, h_blob, h_counts = (pend["val"].numpy(), pend["off"].numpy(), pend["blob"].numpy(),
                                          pend["counts"].numpy())
        need_fix = True
    bounds = np.zeros(nparts + 1, np.int64)
    np.cumsum(h_counts, out=bounds[1:])
    out = {"hi": h_hi, "lo": h_lo, "val": h_val, "key_off": h_off, "key_blob": h_blob, "bounds": bounds}
    if defer:
        out["_downloads"] = flush_downloads(hi.device, wait=False)
        return out
    if need_fix:
        # exact bytewise order inside each partition (long keys sharing a prefix)
        perms = []
        for p in range(nparts):
            a, b = int(bounds[p]), int(bounds[p + 1])
            pp = fix_long_key_order(h_hi[a:b], h_lo[a:b], h_off[a:b + 1], h_blob) if b - a > 1 else None
            perms.append(None if pp is None else pp + a)
        if any(pp is not None for pp in perms):
            gp = np.concatenate([pp if pp is not None else np.arange(int(bounds[p]), int(bounds[p + 1]))
                                 for p, pp in enumerate(perms)])
            out = reorder(out, gp)
    return out


def reorder(cols: dict, perm: np.ndarray) -> dict:
    off = cols["key_off"]
    blob = cols["key_blob"]
    lens = (off[1:] - off[:-1])[perm]
    noff = np.zeros(perm.size + 1, np.int64)
    np.cumsum(lens, out=noff[1:])
    b = blob.tobytes()
    nb = b"".join(b[off[i]:off[i + 1]] for i in perm)
    out = dict(cols)
    out.update(hi=cols["hi"][perm], lo=cols["lo"][perm], val=cols["val"][perm], key_off=noff,
               key_blob=np.frombuffer(nb, dtype=np.uint8))
    return out


def partition_slice(cols: dict, p: int) -> dict:
    a, b = int(cols["bounds"][p]), int(cols["bounds"][p + 1])
    off = cols["key_off"][a:b + 1]
    return {"hi": None if cols["hi"] is None else cols["hi"][a:b],
            "lo": None if cols["lo"] is None else cols["lo"][a:b], "val": cols["val"][a:b],
            "key_off": off - off[0], "key_blob": cols["key_blob"][off[0]:off[-1]]}
