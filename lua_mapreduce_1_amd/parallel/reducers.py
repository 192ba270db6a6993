"""The reduce module's combiner and reducer over value lists grouped on the
device — batched on the GPU when the module says how, per key on the host
otherwise.

Reference contract (/root/reference/mapreduce/job.lua:83-112,198-202,264-284,
task.lua:325): the combiner is the *reduce* module's ``combinerfn``; it runs
map-side on a key's value list whenever the list passes ``MAX_MAP_RESULT``
values and once more per key (with more than one value) at the end of the
map, and its emitted values replace the list; the reducer then runs per key
over the merged lists (skipping singleton lists when the module declares the
three ACI flags).  The general device plane (parallel/generic.py) groups a
rank's values per key in HBM, so here both run over ALL of a rank's lists at
once, in CSR form (``off`` [m + 1], ``val`` [n]):

* ``device_combinerfn(keys, off, val)`` / ``device_reducefn(keys, off, val)``
  — batched torch code (ops/segments.py has the segmented folds, sorts,
  top-k and quantiles); ``keys`` is a :class:`KeyBatch`, ``val`` int64 or
  float64 (the map module's ``device_value_dtype``).  The return value is
  one value per key (a tensor [m]), several (a tuple of tensors [m], or a
  tensor [m, k]) or a variable number (:class:`ValueLists`).  A module whose
  ``combinerfn`` IS its ``reducefn`` (WordCount's reducefn2) uses
  ``device_reducefn`` as its device combiner too;
* otherwise the host ``combinerfn`` / ``reducefn`` run per key over the
  downloaded lists (the last resort: Python per key).

The map-side combine keeps a rank's postings bounded
(:data:`~lua_mapreduce_1_amd.utils.config.Tunables.combine_postings`, the
batched form of ``MAX_MAP_RESULT``) and is applied once more before the
shuffle, so a key ships at most its combined values from each rank.
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch

from .. import ops
from ..ops import segments as S
from ..runtime import codec, modules
from . import recognize as RZ
from . import values as VL
from ..utils.config import TUNABLES


class ValueLists(NamedTuple):
    """A batched reducer's variable-length output: key i emits
    ``val[off[i]:off[i + 1]]``."""
    off: torch.Tensor
    val: torch.Tensor


class KeyBatch:
    """The keys of a batch of value lists: their 128-bit words (``hi``,
    ``lo``, ops/keys.py) and — materialised on first use — their bytes as a
    CSR pair (``key_off`` [m + 1], ``key_blob``)."""

    def __init__(self, hi, lo, rep=None, src=None, key_off=None, key_blob=None):
        self.hi, self.lo, self._rep, self._src = hi, lo, rep, src
        self._off, self._blob = key_off, key_blob

    def __len__(self) -> int:
        return int(self.hi.numel())

    @property
    def device(self):
        return self.hi.device

    def _materialize(self) -> None:
        if self._off is None:
            _, ln = ops.key_meta(self.hi, self.lo, self._rep, self._src, want_part=False)
            self._off, self._blob = ops.gather_key_bytes(self.hi, self.lo, self._rep, self._src, lengths=ln)

    @property
    def key_off(self) -> torch.Tensor:
        self._materialize()
        return self._off

    @property
    def key_blob(self) -> torch.Tensor:
        self._materialize()
        return self._blob

    def strings(self) -> list[str]:
        """The keys as Python strings (host copy)."""
        off = self.key_off.cpu().numpy()
        blob = self.key_blob.cpu().numpy().tobytes()
        return [codec.key_str(blob[off[i]:off[i + 1]]) for i in range(len(self))]


# ---------------------------------------------------------------------------
def _take(v: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    """v[perm] for 8-byte values (GPU: mr_gather_u64 with the sort's int32
    permutation; torch's index kernel was a quarter of the general reducer's
    kernel time, profiles/r4/final_profiles/).  Rows of tuple values ([n, k]):
    v[perm] by rows."""
    if not v.is_cuda or v.element_size() != 8 or v.dim() != 1:
        return v[perm.long()]
    from ..ops import _hip
    src = v.contiguous().view(torch.int64)
    out = torch.empty_like(src)
    p32 = perm.to(torch.int32).contiguous()
    _hip.call("mr_gather_u64", _hip.ptr(src), _hip.ptr(p32), _hip.ptr(out), src.numel(), _hip.stream(v.device))
    return out.view(v.dtype)


def lists_of_postings(slot, pslot, pval, m: int, space: int):
    """A table's postings (key slot, value; emission order) -> the keys' value
    lists in CSR form, key i = the i-th entry of ``slot`` (emission order
    inside a list): (off [m + 1], val)."""
    d = slot.device
    if m == 0:
        return torch.zeros(1, dtype=torch.int64, device=d), pval[:0]
    pos = torch.full((max(space, 1),), m, dtype=torch.int64, device=d)
    pos[slot] = torch.arange(m, dtype=torch.int64, device=d)
    # dropped rows (slot -1) and postings of keys not listed take key index m:
    # the stable sort puts them after every list (no compaction pass)
    if pslot.is_cuda and m < (1 << 31):
        # u32 key indices and their digit histograms in one pass, then the
        # stable u32 radix sort (8 bytes moved per posting and pass, not 12)
        from ..ops import _hip
        from ..ops.primitives import sort_error, sort_keys32
        ps = pslot.to(torch.int64).contiguous()
        k32 = torch.empty(ps.numel(), dtype=torch.int32, device=d)
        ghist = torch.zeros(2048, dtype=torch.int32, device=d)
        _hip.call("mr_posting_keys", _hip.ptr(pos), pos.numel(), _hip.ptr(ps), ps.numel(), m, _hip.ptr(k32),
                  _hip.ptr(ghist), _hip.stream(d))
        bits = (max(1, int(m).bit_length()) + 7) // 8 * 8
        pp, sk = sort_keys32(k32, ghist, bits=bits)
        if sort_error(d):  # a look-back gave up: the checked u64 sort instead
            pp, pr = ops.sort_keys_checked([k32.to(torch.int64)], bits=[bits], return_keys=True)
        else:
            pr = sk
        pv = _take(pval, pp)
    else:
        pr = torch.where(pslot >= 0, pos[pslot.clamp(min=0)], torch.full_like(pslot, m))
        pv = pval
        if pr.numel():
            # stable; the sort hands back its sorted keys (no gather of them) and
            # the values follow the permutation through one u64 gather kernel
            pp, pr = ops.sort_keys_checked([pr], bits=[max(1, int(m).bit_length())], return_keys=True)
            pv = _take(pv, pp)
    # list boundaries of the sorted key indices (no atomics: hot keys are free)
    off = torch.searchsorted(pr, torch.arange(m + 1, dtype=pr.dtype, device=d))
    return off, pv[:int(off[-1])]  # (the sorted-last postings of no key dropped)


def splice(off, val, noff, nval, keep_old):
    """Per key: the old list where ``keep_old`` else the new one -> (off, val)."""
    d = off.device
    lo_, ln = S.lengths(off), S.lengths(noff)
    lens = torch.where(keep_old, lo_, ln)
    roff = S.from_lengths(lens)
    total = int(roff[-1]) if lens.numel() else 0
    if total == 0:
        return roff, val[:0]
    seg = S.ids(roff, total)
    j = torch.arange(total, dtype=torch.int64, device=d) - roff[seg]
    old = keep_old[seg]
    shape = (total,) + tuple(val.shape[1:])
    a = val[(off[seg] + j).clamp(max=max(val.shape[0] - 1, 0))] if val.numel() else \
        torch.zeros(shape, dtype=val.dtype, device=d)
    b = nval[(noff[seg] + j).clamp(max=max(nval.shape[0] - 1, 0))] if nval.numel() else torch.zeros_like(a)
    b = b.to(a.dtype)
    return roff, torch.where(old.unsqueeze(1) if a.dim() == 2 else old, a, b)


def _typed(bits: torch.Tensor, dtype: str) -> torch.Tensor:
    return bits.view(torch.float64) if dtype == "f64" else bits


def _bits(t: torch.Tensor) -> torch.Tensor:
    return t.view(torch.int64) if t.dtype == torch.float64 else t


def _to_list_dtype(v: torch.Tensor, dtype: str, who: str) -> torch.Tensor:
    """A combiner's values in the list dtype (int64 bits of the i64 / f64
    values the lists hold)."""
    if dtype == "f64":
        return v.to(torch.float64).contiguous()
    if v.is_floating_point():
        r = v.round()
        if v.numel() and not bool(torch.equal(r, v)):
            raise TypeError(f"{who} emitted non-integral values into int64 value lists (declare "
                            "device_value_dtype = 'f64' on the map module)")
        v = r
    return v.to(torch.int64).contiguous()


def as_lists(out, m: int, who: str):
    """A batched reducer's return value -> (off, val) CSR."""
    d = None
    if isinstance(out, ValueLists) or (isinstance(out, dict) and "off" in out):
        off, val = (out.off, out.val) if isinstance(out, ValueLists) else (out["off"], out["val"])
        if off.numel() != m + 1:
            raise ValueError(f"{who}: {off.numel()} list offsets for {m} keys (want m + 1)")
        return off.to(torch.int64), val
    if isinstance(out, torch.Tensor):
        if out.dim() == 1:
            out = out.reshape(m, 1) if out.numel() == m else None
        elif out.dim() != 2 or out.shape[0] != m:
            out = None
        if out is None:
            raise ValueError(f"{who}: a tensor result needs one row per key ({m})")
        cols = out
    elif isinstance(out, (tuple, list)) and out and all(isinstance(c, torch.Tensor) for c in out):
        if any(c.numel() != m for c in out):
            raise ValueError(f"{who}: every returned column needs one value per key ({m})")
        dt = torch.float64 if any(c.is_floating_point() for c in out) else torch.int64
        cols = torch.stack([c.reshape(-1).to(dt) for c in out], 1)
    else:
        raise TypeError(f"{who} must return a tensor [m], a tuple of tensors [m], a tensor [m, k] or "
                        f"ValueLists(off, val) (got {type(out).__name__})")
    d = cols.device
    k = cols.shape[1]
    off = torch.arange(m + 1, dtype=torch.int64, device=d) * k
    return off, cols.reshape(-1)


# ---------------------------------------------------------------------------
class ListReducers:
    """The combiner / reducer of a reduce module without ``device_reduce``,
    for value lists of ``dtype`` (``"i64"`` | ``"f64"``, or a
    parallel/values.py spec: tuples, byte strings)."""

    def __init__(self, redmod, dtype="i64"):
        f = modules.field
        self.spec = VL.spec_of(dtype)
        self.dtype = self.spec.dtype
        self.reducefn = f(redmod, "reducefn")
        self.combinerfn = f(redmod, "combinerfn")
        self.device_reducefn = f(redmod, "device_reducefn")
        dc = f(redmod, "device_combinerfn")
        # a host reducer / combiner that is exactly sum / min / max of its
        # values runs batched on the device (parallel/recognize.py)
        self.recognized = {}
        if TUNABLES.recognize_reducers and self.spec.scalar and self.spec.dtype in ("i64", "f64"):
            if self.device_reducefn is None:
                self.device_reducefn = self._recognized("reducefn", self.reducefn)
            if dc is None and self.combinerfn is not None and self.combinerfn is not self.reducefn:
                dc = self._recognized("combinerfn", self.combinerfn)
        if dc is None and self.device_reducefn is not None and self.combinerfn is not None \
                and self.combinerfn is self.reducefn:
            dc = self.device_reducefn  # the combiner is the reducer: so is its batched form
        self.device_combinerfn = dc
        # 'sum' / 'min' / 'max' when the device combiner is a recognised fold:
        # lists of one repeated constant then combine without being built
        # (GenericMap.combine over run-length postings)
        self.combiner_fold = getattr(dc, "recognized", None)
        if self.reducefn is None and self.device_reducefn is None:
            raise ValueError("a reduce module without device_reduce needs a reducefn (or a device_reducefn)")
        self.aci = all(bool(f(redmod, x)) for x in ("associative_reducer", "commutative_reducer",
                                                    "idempotent_reducer"))

    def _recognized(self, name: str, fn):
        op = RZ.recognize(fn)
        fold = RZ.device_fold(op, self.spec.dtype) if op else None
        if fold is not None:
            self.recognized[name] = op
        return fold

    @property
    def has_combiner(self) -> bool:
        return self.combinerfn is not None or self.device_combinerfn is not None

    @property
    def device_reduce(self) -> bool:
        return self.device_reducefn is not None

    # -- the combiner (map side) ---------------------------------------------
    def combine(self, keys: KeyBatch, off: torch.Tensor, val: torch.Tensor, src=None, add_bytes=None):
        """Every key's list with more than one value -> the combiner's values
        (job.lua:198-202); singleton lists are kept.  ``val``: int64 bits of
        the lists' values (rows [n, k] for tuple / byte values, whose bytes
        are spans of ``src``; new byte values go through ``add_bytes``).
        Returns (off, val) in the same form."""
        m = off.numel() - 1
        multi = S.lengths(off) > 1
        if m == 0:
            return off, val
        if not self.spec.scalar:
            if self.device_combinerfn is not None:
                out = self.device_combinerfn(keys, off, VL.to_user(val, self.spec, src))
                noff, nval = self._spec_lists(out, m, "device_combinerfn", add_bytes)
                return splice(off, val, noff, nval, ~multi)
            return self._host_lists_spec(self.combinerfn, keys, off, val, multi, src, add_bytes, "combinerfn")
        if self.device_combinerfn is not None:
            out = self.device_combinerfn(keys, off, _typed(val, self.dtype))
            noff, nval = as_lists(out, m, "device_combinerfn")
            nval = _bits(_to_list_dtype(nval, self.dtype, "device_combinerfn"))
            return splice(off, val, noff, nval, ~multi)
        return self._host_lists(self.combinerfn, keys, off, val, multi, "combinerfn")

    def _host_lists(self, fn, keys: KeyBatch, off, val, sel, who: str):
        """Per selected key on the host: fn(key, values, emit) replaces the
        list (the reference's per-key call)."""
        d = off.device
        o = off.cpu().numpy()
        v = _typed(val, self.dtype).cpu().numpy()
        pick = np.flatnonzero(sel.cpu().numpy())
        if pick.size == 0:
            return off, val
        names = keys.strings()
        lens = np.diff(o)
        outs = []
        for i in pick:
            acc: list = []
            fn(names[i], v[o[i]:o[i + 1]].tolist(), acc.append)
            outs.append(acc)
        new_lens = lens.copy()
        new_lens[pick] = [len(a) for a in outs]
        flat = [x for a in outs for x in a]
        npdt = np.float64 if self.dtype == "f64" else np.int64
        try:
            arr = np.asarray(flat, dtype=np.float64 if self.dtype == "f64" else None)
        except (TypeError, ValueError) as e:
            raise TypeError(f"{who} emitted values that are not numbers: {e}") from None
        if arr.size and arr.dtype != npdt:
            if self.dtype == "i64" and arr.dtype.kind == "f" and np.all(np.floor(arr) == arr):
                arr = arr.astype(np.int64)
            elif self.dtype == "i64" and arr.dtype.kind in "iub":
                arr = arr.astype(np.int64)
            else:
                raise TypeError(f"{who} emitted {arr.dtype} values into {self.dtype} value lists (declare "
                                "device_value_dtype = 'f64' on the map module for real values)")
        arr = arr.astype(npdt, copy=False)
        noff = np.zeros(lens.size + 1, np.int64)
        np.cumsum(new_lens, out=noff[1:])
        res = np.empty(int(noff[-1]), npdt)
        keep = np.ones(lens.size, bool)
        keep[pick] = False
        ki = np.flatnonzero(keep & (lens > 0))
        if ki.size:
            src_idx = np.repeat(o[:-1][ki], lens[ki]) + _ranks(lens[ki])
            dst_idx = np.repeat(noff[:-1][ki], lens[ki]) + _ranks(lens[ki])
            res[dst_idx] = v[src_idx]
        if pick.size and arr.size:
            nl = new_lens[pick]
            dst_idx = np.repeat(noff[:-1][pick], nl) + _ranks(nl)
            res[dst_idx] = arr
        t = torch.from_numpy(res).to(d)
        return torch.from_numpy(noff).to(d), _bits(t)

    def _spec_lists(self, out, m: int, who: str, add_bytes):
        """A batched hook's ValueLists over tuple / byte values -> (off, bits)."""
        if not isinstance(out, ValueLists):
            raise TypeError(f"{who} over {self.spec} values must return ValueLists(off, values)")
        off = out.off.to(torch.int64)
        if off.numel() != m + 1:
            raise ValueError(f"{who}: {off.numel()} list offsets for {m} keys (want m + 1)")
        n = int(off[-1]) if m else 0
        return off, VL.from_user(out.val, self.spec, n, add_bytes, who)

    def _host_lists_spec(self, fn, keys: KeyBatch, off, val, sel, src, add_bytes, who: str):
        """Per selected key on the host over tuple / byte values (the
        reference's per-key combiner call, job.lua:92-96,198-202)."""
        d = off.device
        o = off.cpu().numpy()
        pick = np.flatnonzero(sel.cpu().numpy())
        if pick.size == 0:
            return off, val
        rows = self.spec.rows(val)
        csr = {}
        for j in self.spec.bytes_cols:
            bo, bb = VL.gather_bytes(rows[:, j], src)
            csr[j] = (bo.cpu().numpy(), bb.cpu().numpy())
        py = VL.host_columns(rows.cpu().numpy(), self.spec, csr)
        names = keys.strings()
        lens = np.diff(o)
        outs = []
        for i in pick:
            acc: list = []
            fn(names[i], py[o[i]:o[i + 1]], acc.append)
            outs.append(acc)
        new_lens = lens.copy()
        new_lens[pick] = [len(a) for a in outs]
        noff = np.zeros(lens.size + 1, np.int64)
        np.cumsum(new_lens, out=noff[1:])
        flat = [x for a in outs for x in a]
        nb = VL.host_bits(flat, self.spec, add_bytes, who).reshape(-1, self.spec.width)
        res = np.zeros((int(noff[-1]), self.spec.width), np.int64)
        keep = np.ones(lens.size, bool)
        keep[pick] = False
        ki = np.flatnonzero(keep & (lens > 0))
        host_rows = rows.cpu().numpy()
        if ki.size:
            src_idx = np.repeat(o[:-1][ki], lens[ki]) + _ranks(lens[ki])
            dst_idx = np.repeat(noff[:-1][ki], lens[ki]) + _ranks(lens[ki])
            res[dst_idx] = host_rows[src_idx]
        if pick.size and nb.size:
            nl = new_lens[pick]
            dst_idx = np.repeat(noff[:-1][pick], nl) + _ranks(nl)
            res[dst_idx] = nb
        return torch.from_numpy(noff).to(d), self.spec.storage(torch.from_numpy(res).to(d))

    # -- the reducer (reduce side) ---------------------------------------------
    def reduce_device_cols(self, keys: KeyBatch, off: torch.Tensor, cols: list) -> dict:
        """The batched reducer over tuple / byte-string value lists (``cols``:
        a typed tensor per number column, ByteValues per byte column, as
        order_lists gives them) -> result columns or lists."""
        m = off.numel() - 1
        spec = self.spec
        if spec.width == 1:
            val = cols[0]  # one byte-string column: its ByteValues
        elif not spec.has_bytes and len(set(spec.cols)) == 1:
            val = torch.stack(cols, 1)
        else:
            val = tuple(cols)
        out = self.device_reducefn(keys, off, val)
        if isinstance(out, ValueLists):
            noff = out.off.to(torch.int64)
            if noff.numel() != m + 1:
                raise ValueError(f"device_reducefn: {noff.numel()} list offsets for {m} keys (want m + 1)")
            v = out.val
            if isinstance(v, torch.Tensor) and v.dim() == 1:
                return {"list_off": noff, "list_val": v, "list_typed": True}
            lc = [v[:, j] for j in range(v.shape[1])] if isinstance(v, torch.Tensor) else list(v)
            return {"list_off": noff, "list_cols": lc}
        if isinstance(out, torch.Tensor) and out.dim() == 2:
            rc = [out[:, j] for j in range(out.shape[1])]
        elif isinstance(out, torch.Tensor):
            rc = [out]
        else:
            as_lists(out, m, "device_reducefn")  # validates the shape / type
            rc = list(out)
        rc = [c.reshape(-1) for c in rc]
        if any(c.numel() != m for c in rc):
            raise ValueError(f"device_reducefn: every returned column needs one value per key ({m})")
        return {"cols": rc}

    # -- the reducer (reduce side) ---------------------------------------------
    def reduce_device(self, keys: KeyBatch, off: torch.Tensor, val: torch.Tensor) -> dict:
        """The batched reducer over every key's list -> result columns
        ({"cols": [...]}) or lists ({"list_off", "list_val"}), on the device.
        With the three ACI flags a singleton list is its own result
        (job.lua:264-274) — applied to single-column and list results."""
        m = off.numel() - 1
        out = self.device_reducefn(keys, off, _typed(val, self.dtype))
        single = S.lengths(off) == 1
        if isinstance(out, ValueLists) or (isinstance(out, dict) and "off" in out):
            noff, nval = as_lists(out, m, "device_reducefn")
            if self.aci:
                noff, nval = splice(off, _typed(val, self.dtype).to(nval.dtype), noff, nval, single)
            return {"list_off": noff, "list_val": nval, "list_typed": True}
        if isinstance(out, torch.Tensor) and out.dim() == 2:
            cols = [out[:, j] for j in range(out.shape[1])]
        elif isinstance(out, torch.Tensor):
            cols = [out]
        else:
            as_lists(out, m, "device_reducefn")  # validates the shape / type
            cols = list(out)
        cols = [c.reshape(-1) for c in cols]
        if any(c.numel() != m for c in cols):
            raise ValueError(f"device_reducefn: every returned column needs one value per key ({m})")
        if self.aci and len(cols) == 1 and m:
            c = cols[0]
            cols = [torch.where(single, S.first(off, _typed(val, self.dtype)).to(c.dtype), c)]
        return {"cols": cols}


def _ranks(lens: np.ndarray) -> np.ndarray:
    """0, 1, .., lens[0]-1, 0, 1, .., lens[1]-1, ..."""
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    starts = np.zeros(lens.size, np.int64)
    np.cumsum(lens[:-1], out=starts[1:])
    return np.arange(total, dtype=np.int64) - np.repeat(starts, lens)
