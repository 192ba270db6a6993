"""Dense-tensor values on the device: the SPMD engine's tensor plane
(``device_reduce = "tensor_sum"``).

The reference's iterative DP-SGD example emits, per map job, one serialised
gradient per weight name (/root/reference/mapreduce/examples/APRIL-ANN/
common.lua:85-104), partitions the names by a byte sum (:106-109), sums them
per name in the reduce jobs (:112-137) and hands the sums to finalfn, which
steps the optimizer and loops (:144-202).  Keys are few and values are
large fixed-width vectors — the shape of a gradient all-reduce — so this
plane keeps them as fp32 tensors in HBM end to end:

* the map module declares its keys and their sizes,
  ``device_tensor_layout = {"w1": 32768, ...}`` (or a function of no
  arguments returning it), and its ``device_mapfn`` calls
  ``emit.tensor(key, t)`` — t is added into the key's slice of one per-rank
  accumulator (the map-side combiner: the values of a key are summed as they
  are emitted) — or writes into ``emit.accumulator(key)`` in place;
* the layout groups the keys by the rank that owns their partition
  (``partitionfn(key)`` -> p, owned by rank p % W, as every plane does) into
  W equal, padded chunks, so the shuffle + reduce is ONE reduce-scatter
  (RCCL over xGMI): rank r receives the sums of exactly the keys it owns —
  the reduce jobs of the partitions present (server.lua:279-326);
* one all-gather then gives every rank every key's sum for finalfn; a
  module's ``device_finalfn(res, engine)`` runs on every rank over
  ``res.tensors`` (key -> device tensor), so replicated state (the model)
  is updated identically everywhere with no host copy of the values; a host
  ``finalfn`` gets (key, [numpy array]) pairs from rank 0.

On gloo (CPU tests) the reduce-scatter and the all-gather are one all-reduce of
the buffer (gloo has neither primitive on tensors).
"""
from __future__ import annotations

import sys
import time
import traceback

import numpy as np
import torch

from .. import utils
from ..runtime import modules
from ..utils import STATUS
from ..utils import trace
from . import dist as D

TENSOR_OPS = ("tensor_sum",)
_ALIGN = 64  # floats: chunk boundaries on 256-byte lines
FAILED_KEY = "__failed_maps__"


class TensorEmitter:
    """``emit`` of a tensor-plane map."""

    def __init__(self, plane: "TensorPlane"):
        self.plane = plane

    @property
    def device(self):
        return self.plane.eng.device

    def accumulator(self, key) -> torch.Tensor:
        """The fp32 view this rank sums ``key``'s values into (write or add in
        place; it is zeroed at the start of every iteration)."""
        return self.plane.view(self.plane.buf, key)

    def tensor(self, key, t) -> None:
        a = self.accumulator(key)
        t = torch.as_tensor(t, device=a.device).reshape(-1)
        if t.numel() != a.numel():
            raise ValueError(f"emit.tensor({key!r}): {t.numel()} values, the layout declares {a.numel()}")
        a.add_(t.to(torch.float32))

    def __call__(self, key, value) -> None:
        self.tensor(key, value)

    def error_word(self):
        return None


class TensorResult:
    """The iteration's sums: ``tensors`` (key -> fp32 device tensor, every
    key, on every rank after the all-gather) and the reference's per
    partition view of this rank's keys (``partitions``, host numpy)."""

    def __init__(self):
        self.result_names: dict[int, str] = {}
        self.map_jobs: list = []
        self.red_jobs: list = []
        self.timings: dict[str, float] = {}
        self.distinct_keys = 0
        self.total_value = 0
        self.failed_reduces = 0
        self.tensors: dict = {}
        self._failed_view = None
        self._parts = None
        self._materialize = None

    @property
    def failed_maps(self) -> int:
        """Map jobs FAILED on any rank (summed in the reduce with the values)."""
        return int(self._failed_view.item()) if self._failed_view is not None else 0

    @property
    def partitions(self) -> dict:
        if self._parts is None:
            self._parts = self._materialize() if self._materialize is not None else {}
        return self._parts


class TensorPlane:
    def __init__(self, eng):
        self.eng = eng
        lay = modules.field(eng.mapmod, "device_tensor_layout")
        if callable(lay):
            lay = lay()
        if not lay:
            raise ValueError("device_reduce 'tensor_sum' needs device_tensor_layout = {key: size, ...} on the map "
                             "module")
        part = modules.field(eng.partmod, "partitionfn")
        W = eng.world
        keys = {}
        for k, n in dict(lay).items():
            p = int(part(k))
            if p != part(k) or p < 0:
                raise ValueError(f"partitionfn({k!r}) = {part(k)!r}: partitions are integers >= 0")
            keys[k] = (p, int(n))
        if not eng.params.get("num_partitions"):
            # result.P<NN> names cover the partitions the keys fall in
            eng.nparts = max(eng.nparts, max(p for p, _n in keys.values()) + 1)
        # the failed-map count rides in the buffer (owned by rank 0)
        keys[FAILED_KEY] = (-1, 1)
        self.part_of = {k: v[0] for k, v in keys.items()}
        owner = {k: (p % W if p >= 0 else 0) for k, (p, _n) in keys.items()}
        per_rank: list = [[] for _ in range(W)]
        for k in sorted(keys, key=lambda k: (keys[k][0], str(k))):
            per_rank[owner[k]].append(k)
        sizes = [sum(keys[k][1] for k in ks) for ks in per_rank]
        C = max(_ALIGN, -(-max(sizes) // _ALIGN) * _ALIGN)
        self.chunk = C
        self.offset: dict = {}
        for r, ks in enumerate(per_rank):
            o = r * C
            for k in ks:
                self.offset[k] = (o, keys[k][1])
                o += keys[k][1]
        self.owned = per_rank[eng.rank]
        d = eng.device
        self.buf = torch.zeros(W * C, dtype=torch.float32, device=d)   # this rank's map sums (all keys)
        self.full = torch.zeros(W * C, dtype=torch.float32, device=d)  # every key's global sum
        self.emitter = TensorEmitter(self)

    def view(self, t: torch.Tensor, key) -> torch.Tensor:
        if key not in self.offset:
            raise KeyError(f"key {key!r} is not in device_tensor_layout")
        o, n = self.offset[key]
        return t[o:o + n]

    # -- shuffle + reduce: reduce-scatter by partition, then the all-gather ------------
    def _reduce_scatter_gather(self) -> None:
        eng = self.eng
        W, C = eng.world, self.chunk
        if W == 1 and not eng.force_shuffle:
            self.full.copy_(self.buf)
            return
        import torch.distributed as tdist
        if D._is_gloo(eng.group):
            # gloo: the same sums through an all-reduce of the buffer (gloo has no
            # reduce-scatter / all-gather into a tensor)
            h = self.buf.cpu()
            tdist.all_reduce(h, group=eng.group)
            self.full.copy_(h)
            return
        r = eng.rank
        mine = self.full[r * C:(r + 1) * C]
        with trace.range("mr.tensor.reduce_scatter"):
            tdist.reduce_scatter_tensor(mine, self.buf, group=eng.group)  # rank r: the sums of its partitions
        with trace.range("mr.tensor.all_gather"):
            tdist.all_gather_into_tensor(self.full, mine.clone(), group=eng.group)

    # -- one iteration -------------------------------------------------------------------
    def run_iteration(self, prefetch_next=None, lookahead=None) -> TensorResult:
        from .planes import _records, _result_jobs
        eng = self.eng
        eng.iteration += 1
        res = TensorResult()
        T = res.timings
        t0 = time.time()
        jobs = eng._jobs()
        j0, j1 = eng._assign(jobs)
        recs = _records(eng, jobs, j0, j1, t0)
        res.map_jobs = recs
        dmap = eng.dmap
        self.buf.zero_()
        failed = 0
        with trace.range("mr.tensor.map"):
            for j in range(j0, j1):
                r = recs[j]
                ta, c0 = time.time(), time.process_time()
                snap = self.buf.clone() if j1 - j0 > 1 else None
                for attempt in range(utils.MAX_JOB_RETRIES):
                    try:
                        dmap(jobs[j][0], jobs[j][1], self.emitter)
                        r.status = STATUS.WRITTEN
                        break
                    except Exception:  # noqa: BLE001  (BROKEN -> retried; FAILED after MAX_JOB_RETRIES)
                        r.repetitions += 1
                        r.status = STATUS.BROKEN
                        sys.stderr.write("# rank %d map job %r attempt %d failed:\n%s" % (
                            eng.rank, jobs[j][0], attempt + 1, traceback.format_exc()))
                        if snap is not None:
                            self.buf.copy_(snap)  # drop the failed attempt's partial sums
                        else:
                            self.buf.zero_()
                if r.status != STATUS.WRITTEN:
                    r.status = STATUS.FAILED
                    failed += 1
                r.written = time.time()
                r.real_time, r.cpu_time = r.written - ta, time.process_time() - c0
        self.view(self.buf, FAILED_KEY).fill_(float(failed))
        eng._maybe_inject_fault("shuffle")
        t1 = time.time()
        T["map"] = t1 - t0
        self._reduce_scatter_gather()
        T["shuffle"] = time.time() - t1
        t2 = time.time()
        res.tensors = {k: self.view(self.full, k) for k in self.offset if k != FAILED_KEY}
        counts = [0] * eng.nparts
        for k in self.owned:
            p = self.part_of[k]
            if 0 <= p < eng.nparts:
                counts[p] += 1
        _result_jobs(eng, res, counts, t1)
        res.distinct_keys = len(self.owned) - (FAILED_KEY in self.owned)
        res._failed_view = self.view(self.full, FAILED_KEY)
        res._materialize = lambda: self._host_parts(res)
        T["reduce"] = time.time() - t2
        T["iteration"] = time.time() - t0
        return res

    def _host_parts(self, res) -> dict:
        """This rank's partitions on the host: {p: {"keys": [...], "values": [np.ndarray]}}."""
        out: dict = {}
        for k in self.owned:
            p = self.part_of[k]
            if p < 0:
                continue
            e = out.setdefault(p, {"keys": [], "values": []})
            e["keys"].append(k)
            e["values"].append(res.tensors[k].detach().cpu().numpy())
        return out
