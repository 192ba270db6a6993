"""Inverted-index primitives (HIP kernels in ``csrc/hip/invidx.hip``; NumPy /
torch on CPU tensors).

A posting is ONE 64-bit key ``[dest | word id | doc]`` (see invidx.hip): the
map emits one per token, a radix sort groups them by destination rank, word
and document, and a compaction drops repeats of a word inside one line.
Word ids are the slots of an HBM hash table on the GPU (dense ids from
``np.unique`` on the CPU); the table also keeps each word's (hi, lo, rep) so key
bytes are materialised only for the final words.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _hip
from . import keys as K
from .primitives import HashTable, _t64, _u64, exclusive_scan, sort_keys

# bytes per ii_map workgroup: ONE 8 KiB tile (1 workgroup per CU fits; 8/16/32/64 KiB
# measured 10.5 / 11.5 / 12.4 / 15.5 ms per build: more, shorter workgroups balance the
# CUs and their LDS tables fill less), MR_II_CHUNK for A/B runs
CHUNK = int(os.environ.get("MR_II_CHUNK", 8 * 1024))


def bits_for(n: int) -> int:
    """Bits needed to hold values 0..n-1 (>= 1)."""
    return max(1, int(max(n, 1) - 1).bit_length())


class Vocab:
    """Word ids of one rank: ``hi/lo/rep`` indexed by id, ``id_bits``."""

    def __init__(self, device, capacity: int = 1 << 21):
        self.device = torch.device(device)
        if self.device.type == "cuda":
            self.table = HashTable(capacity, self.device, "sum")
            self.id_bits = bits_for(self.table.cap)
        else:
            self.table = None
            self.id_bits = 1
            self.hi = self.lo = self.rep = torch.zeros(0, dtype=torch.int64)

    @property
    def overflowed(self) -> bool:
        return self.table is not None and int(self.table.ctrl[1].item()) != 0

    def arrays(self):
        if self.table is not None:
            # (the table's hi / lo / rep are strided fields of its key records)
            return self.table.hi.contiguous(), self.table.lo.contiguous(), self.table.rep.contiguous()
        return self.hi, self.lo, self.rep

    def reset(self) -> None:
        if self.table is not None:
            self.table.reset()

    # -- CPU helpers --------------------------------------------------------------
    def _assign_cpu(self, hi: np.ndarray, lo: np.ndarray, rep: np.ndarray, src=None) -> np.ndarray:
        """Dense ids for (hi, lo) (first occurrence keeps its rep); long keys
        that collide on (hi, lo) get different ids when their bytes differ."""
        keys = np.empty(hi.size, dtype=[("h", "<u8"), ("l", "<u8"), ("d", "<i8")])
        keys["h"], keys["l"], keys["d"] = hi, lo, 0
        long_ = (lo & np.uint64(0xFF)) == np.uint64(K.LONG_MARK)
        if long_.any() and src is not None:
            sb = src.numpy() if isinstance(src, torch.Tensor) else np.asarray(src)
            ids: dict = {}
            ru = rep.view(np.uint64)
            for i in np.flatnonzero(long_):
                o, ln = int(ru[i]) >> K.REP_LEN_BITS, int(ru[i]) & K.REP_LEN_MASK
                keys["d"][i] = ids.setdefault(sb[o:o + ln].tobytes(), len(ids) + 1)
        uk, first, inv = np.unique(keys, return_index=True, return_inverse=True)
        self.hi = _t64(uk["h"].copy())
        self.lo = _t64(uk["l"].copy())
        self.rep = _t64(rep[first])
        self.id_bits = bits_for(uk.size)
        return inv.astype(np.int64)


def _chunk_bases(text: torch.Tensor, nbytes: int, s):
    """Per map chunk: first line (exclusive scan of newline counts) and first
    token (exclusive scan of token counts, + their total) — the map kernel
    writes every posting at its text-order index."""
    d = text.device
    nchunks = max(1, (nbytes + CHUNK - 1) // CHUNK)
    cnt = torch.empty((2, nchunks), dtype=torch.int32, device=d)
    _hip.call("mr_count_newlines", _hip.ptr(text), nbytes, CHUNK, _hip.ptr(cnt[0]), _hip.ptr(cnt[1]), s)
    lbase, _ = exclusive_scan(cnt[0])
    tbase, ttot = exclusive_scan(cnt[1])
    return lbase, tbase, ttot, cnt[1]


def map_postings(text: torch.Tensor, vocab: Vocab, doc_bits: int, rep_base: int = 0):
    """Posting keys ``id << doc_bits | line`` of every token of ``text``, in
    text order (so in line order) -> int64 tensor.  ``line`` = newlines before
    the token."""
    nbytes = text.numel()
    if text.is_cuda:
        d = text.device
        s = _hip.stream(d)
        base, tbase, ttot, tcnt = _chunk_bases(text, nbytes, s)
        cap = nbytes // 2 + 2  # tokens are separated by >= 1 whitespace byte
        out = torch.empty(cap, dtype=torch.int64, device=d)
        counter = torch.zeros(1, dtype=torch.int64, device=d)
        err = torch.zeros(1, dtype=torch.int32, device=d)
        t = vocab.table
        _hip.call("mr_ii_map", _hip.ptr(text), nbytes, CHUNK, rep_base, _hip.ptr(base), _hip.ptr(tbase),
                  _hip.ptr(tcnt), *t._gtab(), t.cap, doc_bits, _hip.ptr(out), _hip.ptr(counter), cap, _hip.ptr(err), s)
        _hip.call("mr_ii_advance", _hip.ptr(counter), _hip.ptr(ttot), s)
        n, e = torch.cat([counter, err.to(torch.int64)]).tolist()
        if e & 2:
            raise RuntimeError("inverted index map: a chunk's tokens differ from its reserved count")
        if e:
            raise RuntimeError("inverted index map: posting buffer overflow")
        if vocab.overflowed:
            raise RuntimeError("inverted index map: vocabulary table overflow (raise capacity)")
        return out[:n]
    buf = text.numpy()
    starts, lens = K.token_spans(buf)
    hi, lo = K.span_keys(buf, starts, lens)
    rep = ((starts.astype(np.uint64) + np.uint64(rep_base)) << np.uint64(K.REP_LEN_BITS)) | \
        np.minimum(lens, K.REP_LEN_MASK).astype(np.uint64)
    ids = vocab._assign_cpu(hi, lo, rep.view(np.int64), buf)
    nl = np.flatnonzero(buf == 10)
    line = np.searchsorted(nl, starts, side="left").astype(np.int64)
    return torch.from_numpy((ids << doc_bits) | line)


class PostingSink:
    """Device output of map_postings_chunk: one posting buffer and counter
    shared by several launches (chunks of one rank's text, mapped as their
    host->HBM copies land)."""

    def __init__(self, device, nbytes: int):
        self.cap = nbytes // 2 + 2  # tokens are separated by >= 1 whitespace byte
        self.out = torch.empty(self.cap, dtype=torch.int64, device=device)
        self.ctrl = torch.zeros(2, dtype=torch.int64, device=device)  # [count, error]

    def reset(self) -> None:
        self.ctrl.zero_()

    def ctrl_snapshot(self) -> torch.Tensor:
        """Posting count before a chunk's map (device copy, no sync)."""
        return self.ctrl[:1].clone()

    def ctrl_restore(self, snap: torch.Tensor) -> None:
        """Drop the postings written since ``snap`` (a map attempt that raised)."""
        self.ctrl[:1].copy_(snap)

    def finish(self, vocab: "Vocab") -> torch.Tensor:
        n, e = self.ctrl.tolist()  # the one host synchronisation of the map phase
        if e & 2:
            raise RuntimeError("inverted index map: a chunk's tokens differ from its reserved count")
        if e:
            raise RuntimeError("inverted index map: posting buffer overflow")
        if vocab.overflowed:
            raise RuntimeError("inverted index map: vocabulary table overflow (raise capacity)")
        return self.out[:n]


def map_postings_chunk(text: torch.Tensor, a: int, b: int, line_base: int, vocab: Vocab, doc_bits: int,
                       sink: PostingSink) -> None:
    """GPU: postings of text[a:b] (a split-aligned piece of a rank's text) into
    ``sink`` after the postings already there, in text order (pieces are
    mapped in text order, so the sink stays in line order); ``line_base`` =
    newlines of the rank's text before byte a.  Line and token bases come from
    the piece's own counts (one count launch, two scans)."""
    d = text.device
    s = _hip.stream(d)
    piece = text[a:b]
    nbytes = piece.numel()
    if nbytes == 0:
        return
    base, tbase, ttot, tcnt = _chunk_bases(piece, nbytes, s)
    if line_base:
        base.add_(line_base)
    t = vocab.table
    _hip.call("mr_ii_map", _hip.ptr(piece), nbytes, CHUNK, a, _hip.ptr(base), _hip.ptr(tbase), _hip.ptr(tcnt),
              *t._gtab(), t.cap, doc_bits, _hip.ptr(sink.out), _hip.ptr(sink.ctrl[:1]), sink.cap,
              _hip.ptr(sink.ctrl[1:]), s)
    _hip.call("mr_ii_advance", _hip.ptr(sink.ctrl[:1]), _hip.ptr(ttot), s)


def sort_unique(keys: torch.Tensor, bits: int, from_bit: int = 0, runs: bool = False) -> torch.Tensor:
    """Sorted distinct posting keys (keys < 2^bits, bits <= 63).  ``from_bit``
    (a multiple of 8): the keys are already in order of their bits below it
    (postings in text order: line order), so a stable sort of the bits above
    is enough.  ``runs``: consecutive keys share the sorted digits (a hint
    for the digit histograms: word bits of text-order postings do not)."""
    n = keys.numel()
    if keys.is_cuda:
        if n == 0:
            return keys
        d = keys.device
        s = _hip.stream(d)
        # keys-only radix sort (no permutation carried), then the fused
        # two-pass unique (per-tile head counts -> scan -> scatter)
        _, sk = sort_keys([keys], bits=[bits], return_keys=True, keys_only=True, runs=runs, from_bit=from_bit)
        tiles = int(_hip.lib().mr_ii_unique_tiles(n))
        tc = torch.empty(tiles, dtype=torch.int32, device=d)
        _hip.call("mr_ii_unique_count", _hip.ptr(sk), n, _hip.ptr(tc), s)
        off, total = exclusive_scan(tc)
        m = int(total.item())
        out = torch.empty(m, dtype=torch.int64, device=d)
        _hip.call("mr_ii_unique_scatter", _hip.ptr(sk), n, _hip.ptr(off), _hip.ptr(out), s)
        return out
    return torch.unique(keys)


def group_words(keys: torch.Tensor, doc_bits: int, id_bits: int, doc_base: int = 0, unique: bool = True):
    """Sorted posting keys -> (word ids int64[nw], word starts int64[nw+1],
    docs int32[m]): :func:`split_words` of the distinct keys (``unique``) or
    of all of them.  GPU: one count pass + one scatter pass over the keys
    (csrc/hip/invidx.hip gw_*), no per-posting flag arrays."""
    n = keys.numel()
    if not keys.is_cuda:
        return split_words(torch.unique(keys) if unique else keys, doc_bits, id_bits, doc_base)
    d = keys.device
    if n == 0:
        z = torch.zeros(0, dtype=torch.int64, device=d)
        return z, torch.zeros(1, dtype=torch.int64, device=d), torch.zeros(0, dtype=torch.int32, device=d)
    s = _hip.stream(d)
    tiles = int(_hip.lib().mr_ii_unique_tiles(n))
    tc = torch.empty(2 * tiles, dtype=torch.int32, device=d)
    _hip.call("mr_ii_group_count", _hip.ptr(keys), n, doc_bits, 1 if unique else 0, _hip.ptr(tc), s)
    ok, nk = exclusive_scan(tc[:tiles])
    oh, nh = exclusive_scan(tc[tiles:])
    off = torch.cat([ok, oh]).contiguous()
    m, nw = (int(x) for x in torch.stack([nk.reshape(()), nh.reshape(())]).tolist())  # one synchronisation
    docs = torch.empty(m, dtype=torch.int32, device=d)
    wid = torch.empty(nw, dtype=torch.int64, device=d)
    wstart = torch.empty(nw + 1, dtype=torch.int64, device=d)
    wstart[nw:].fill_(m)
    _hip.call("mr_ii_group_scatter", _hip.ptr(keys), n, doc_bits, int(doc_base), (1 << id_bits) - 1,
              1 if unique else 0, _hip.ptr(off), _hip.ptr(docs), _hip.ptr(wid), _hip.ptr(wstart), s)
    return wid, wstart, docs


def split_words(ukeys: torch.Tensor, doc_bits: int, id_bits: int, doc_base: int = 0):
    """Sorted unique posting keys -> (word ids int64[nw], word starts
    int64[nw+1], docs int32[n]).  Words are runs of equal ``key >> doc_bits``
    (destination bits included, so a word never spans two destinations).
    CPU; the GPU groups sorted keys with :func:`group_words`."""
    n = ukeys.numel()
    id_mask = (1 << id_bits) - 1
    wk = ukeys >> doc_bits
    flags = torch.ones(n, dtype=torch.bool)
    if n > 1:
        flags[1:] = wk[1:] != wk[:-1]
    starts = torch.nonzero(flags).flatten()
    wid = wk[starts] & id_mask
    wstart = torch.cat([starts, torch.tensor([n])]).to(torch.int64)
    docs = ((ukeys & ((1 << doc_bits) - 1)) + doc_base).to(torch.int32)
    return wid, wstart, docs


def add_dest(keys: torch.Tensor, dest_of_id: torch.Tensor, doc_bits: int, id_bits: int) -> int:
    """keys |= dest[id(key)] << (id_bits + doc_bits) in place; returns the shift."""
    shift = id_bits + doc_bits
    if keys.is_cuda:
        _hip.call("mr_ii_add_dest", _hip.ptr(keys), keys.numel(), _hip.ptr(dest_of_id.to(torch.int32).contiguous()),
                  doc_bits, (1 << id_bits) - 1, shift, _hip.stream(keys.device))
        return shift
    ids = (keys >> doc_bits) & ((1 << id_bits) - 1)
    keys |= dest_of_id.to(torch.int64)[ids] << shift
    return shift


def insert_ids(vocab: Vocab, hi: torch.Tensor, lo: torch.Tensor, rep: torch.Tensor,
               src: torch.Tensor | None = None) -> torch.Tensor:
    """Ids of (hi, lo) in ``vocab`` (inserting new words) -> int64.  ``src``:
    the bytes the rep words index (exact identity of long keys)."""
    n = hi.numel()
    if hi.is_cuda:
        t = vocab.table
        out = torch.empty(n, dtype=torch.int64, device=hi.device)
        _hip.call("mr_ii_insert_slots", *t._gtab(), t.cap, _hip.ptr(hi), _hip.ptr(lo), _hip.ptr(rep), n,
                  _hip.ptr(out), _hip.ptr(src), _hip.stream(hi.device))
        if vocab.overflowed:
            raise RuntimeError("inverted index reduce: vocabulary table overflow")
        return out
    return torch.from_numpy(vocab._assign_cpu(_u64(hi), _u64(lo), rep.numpy(), src))


def seg_gather(perm: torch.Tensor, old_start: torch.Tensor, new_off: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """Posting lists reordered by a word permutation: word i of the output is
    word perm[i] of the input (``old_start`` = input word starts, nw_in+1
    entries; ``new_off`` = output offsets, nw+1 entries).  ``perm`` may select
    a subset of the words (a reduce round): the output then holds only their
    lists.  int32 postings."""
    nw = perm.numel()
    nw_in = old_start.numel() - 1
    n_src = src.numel()
    n = n_src if nw == nw_in else (int(new_off[-1]) if nw else 0)
    if src.is_cuda:
        out = torch.empty(n, dtype=torch.int32, device=src.device)
        p32 = perm.to(torch.int32).contiguous()
        _hip.call("mr_ii_seg_gather", _hip.ptr(p32), _hip.ptr(old_start.contiguous()), _hip.ptr(new_off.contiguous()),
                  nw, n, nw_in, n_src, _hip.ptr(src), _hip.ptr(out), _hip.stream(src.device))
        return out
    if nw == 0 or n == 0:
        return src[:0].clone()
    p = perm.long()
    lens = (old_start[1:] - old_start[:-1])[p]
    idx = torch.cat([torch.arange(int(old_start[int(w)]), int(old_start[int(w)]) + int(ln))
                     for w, ln in zip(p.tolist(), lens.tolist())])
    return src[idx]
