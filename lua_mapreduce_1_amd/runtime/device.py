"""Device (HBM) data plane of a map/reduce job.

A map module opts in by defining ``device_mapfn(key, value, emit)``; ``emit``
is a :class:`DeviceEmitter` whose calls feed HBM-resident kernels instead of
Python dicts:

* ``emit.words(text_u8)`` — every whitespace token of a byte tensor with value
  1, through the fused tokenize + exact-key + LDS-combine kernel (K1-K5);
* ``emit.pairs(hi, lo, vals, rep=None, src=None)`` — a batch of (key, value)
  pairs already encoded as 128-bit keys (ops.keys);
* ``emit(key, value)`` — one host pair (buffered, inserted in one batch).

Values are int64 and are folded at insert time with the reduce module's
``device_reduce`` op (``"sum" | "min" | "max"``), i.e. the combiner of
job.lua:92-96,198-202 runs inside the hash table.  Partitioning uses the
partition module's ``device_partition = ("fnv1", N)`` (exact FNV-1 of the key
bytes mod N, examples/WordCount/partitionfn.lua) or, failing that, the host
``partitionfn`` once per distinct key.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from ..ops import keys as K


def default_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class DeviceMapContext:
    def __init__(self, device=None, op: str = "sum", capacity: int = 1 << 20):
        self.device = torch.device(device) if device is not None else default_device()
        self.op = op
        self.capacity = capacity
        self.table = ops.HashTable(capacity, device=self.device, op=op)
        self.sources: list[torch.Tensor] = []
        self.base = 0
        self.host_pairs: list[tuple[bytes, int]] = []
        self.emit = DeviceEmitter(self)

    def add_source(self, t: torch.Tensor) -> int:
        b = self.base
        self.sources.append(t)
        self.base += t.numel()
        return b

    def source(self) -> torch.Tensor | None:
        if not self.sources:
            return None
        if len(self.sources) == 1:
            return self.sources[0]
        return torch.cat(self.sources)

    def flush_host_pairs(self) -> None:
        if not self.host_pairs:
            return
        blob = b"".join(k for k, _ in self.host_pairs)
        base = self.add_source(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.device))
        his, los, reps, off = [], [], [], 0
        for k, _ in self.host_pairs:
            h, l_ = K.pack_key(k)
            his.append(h)
            los.append(l_)
            reps.append(K.make_rep(base + off, len(k)))
            off += len(k)
        t = lambda a: torch.from_numpy(np.array(a, dtype=np.uint64).view(np.int64)).to(self.device)  # noqa: E731
        vals = torch.tensor([v for _, v in self.host_pairs], dtype=torch.int64, device=self.device)
        self.table.insert(t(his), t(los), vals, t(reps))
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
        if text.device != self.ctx.device:
            text = text.to(self.ctx.device, non_blocking=True)
        base = self.ctx.add_source(text)
        self.ctx.table.wordcount_map(text, rep_base=base)

    def pairs(self, hi, lo, vals=None, rep=None, src: torch.Tensor | None = None) -> None:
        add = 0
        if src is not None:
            add = self.ctx.add_source(src.to(self.ctx.device))
        self.ctx.table.insert(hi, lo, vals, rep, rep_add=add)

    def __call__(self, key, value=1) -> None:
        if isinstance(key, str):
            key = key.encode("utf-8", "surrogateescape")
        elif not isinstance(key, bytes):
            key = str(key).encode()
        self.ctx.host_pairs.append((key, int(value)))


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
    """
    n = hi.size
    perm = np.arange(n)
    if n == 0:
        return perm
    is_long = (lo & np.uint64(0xFF)) == np.uint64(0xFF)
    if not is_long.any():
        return perm
    starts = np.flatnonzero(np.concatenate([[True], hi[1:] != hi[:-1]]))
    ends = np.concatenate([starts[1:], [n]])
    has_long = np.add.reduceat(is_long.astype(np.int64), starts) > 0
    b = blob.tobytes() if isinstance(blob, np.ndarray) else bytes(blob)
    for s, e in zip(starts[has_long], ends[has_long]):
        if e - s > 1:
            idx = list(range(s, e))
            idx.sort(key=lambda i: b[off[i]:off[i + 1]])
            perm[s:e] = idx
    return perm


def finalize(hi, lo, val, rep, src, nparts: int, partition_module=None, part: torch.Tensor | None = None):
    """Partition, sort by (partition, key) and materialise key bytes.

    Returns a dict of host numpy arrays: hi, lo, val, key_off, key_blob and
    ``bounds`` (partition p occupies rows bounds[p]:bounds[p+1]).
    """
    n = hi.numel()
    if part is None:
        part = partition_of(hi, lo, rep, src, nparts, partition_module)
    perm = ops.sort_keys([part.to(torch.int64), hi, lo], bits=[max(8, int(nparts - 1).bit_length()), 64, 64])
    perm = perm.long()
    hi, lo, val, rep, part = hi[perm], lo[perm], val[perm], rep[perm], part[perm]
    off, blob = ops.gather_key_bytes(hi, lo, rep, src)
    counts = ops.bincount(part, nparts).cpu().numpy() if n else np.zeros(nparts, np.int64)
    bounds = np.zeros(nparts + 1, np.int64)
    np.cumsum(counts, out=bounds[1:])
    out = {"hi": hi.cpu().numpy().view(np.uint64), "lo": lo.cpu().numpy().view(np.uint64),
           "val": val.cpu().numpy(), "key_off": off.cpu().numpy(), "key_blob": blob.cpu().numpy(),
           "bounds": bounds}
    # exact bytewise order inside each partition (long keys)
    perms = []
    for p in range(nparts):
        a, b = int(bounds[p]), int(bounds[p + 1])
        if b - a > 1:
            pp = fix_long_key_order(out["hi"][a:b], out["lo"][a:b], out["key_off"][a:b + 1] - 0, out["key_blob"])
            perms.append(pp + a)
        else:
            perms.append(np.arange(a, b))
    gp = np.concatenate(perms) if perms else np.zeros(0, np.int64)
    if not np.array_equal(gp, np.arange(n)):
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
    return {"hi": cols["hi"][a:b], "lo": cols["lo"][a:b], "val": cols["val"][a:b], "key_off": off - off[0],
            "key_blob": cols["key_blob"][off[0]:off[-1]]}
