"""SPMD inverted-index build: word -> sorted list of the lines it occurs in.

The BASELINE.json "inverted-index build on the same corpus shape" workload
(variable-length emit, shuffle skew).  As a MapReduce job: the map emits
(word, line) for every token, the partitioner is FNV-1(word) mod R, the reduce
concatenates and de-duplicates the line lists (the segmented concat of the
reference's reducer, SURVEY.md §2.2 K8, over the k-way merge K9).

MI355X pipeline, one rank per GPU, all of it in HBM:
  1. the rank's contiguous block of splits is copied host(pinned) -> HBM once;
  2. ``ii_map`` (HIP) turns every token into one 64-bit posting key
     ``word id << doc_bits | line`` — word ids are HBM hash-table slots, found
     through a per-workgroup LDS table so a chunk's vocabulary costs one HBM
     insert per distinct word;
  3. (W > 1) the destination rank ``FNV-1(word) % R % W`` is OR-ed into the top
     bits, so ONE radix sort groups by destination, word and line, and a
     compaction drops a word's repeats within a line;
  4. (W > 1) the shuffle is three ``all_to_all_single`` calls (word records,
     key bytes, line ids) after one count exchange — RCCL over xGMI;
     receivers merge the words of all sources in a second hash table and sort
     ``(word id << 32 | line)`` (sources hold disjoint line ranges);
  5. the index stays resident: per word the key bytes (offsets + blob), the
     posting offsets and the int32 line ids, plus the word's partition.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import ops
from ..ops import _hip
from ..ops import invidx as II
from ..ops.keys import REP_LEN_BITS
from . import dist as D
from .spmd import SplitStore, assign_contiguous


class IndexShard:
    """The words a rank owns and their posting lists (device or CPU tensors)."""

    def __init__(self, hi, lo, key_off, key_blob, post_off, docs, part):
        self.hi, self.lo = hi, lo
        self.key_off, self.key_blob = key_off, key_blob
        self.post_off, self.docs, self.part = post_off, docs, part

    @property
    def num_words(self) -> int:
        return int(self.hi.numel())

    @property
    def num_postings(self) -> int:
        return int(self.docs.numel())

    def to_host(self) -> dict:
        ko = self.key_off.cpu().numpy()
        kb = self.key_blob.cpu().numpy().tobytes()
        po = self.post_off.cpu().numpy()
        dc = self.docs.cpu().numpy()
        return {kb[ko[i]:ko[i + 1]]: dc[po[i]:po[i + 1]].tolist() for i in range(self.num_words)}

    def partitions(self) -> dict[int, list[int]]:
        """partition -> word indices (the ``result.P<NN>`` grouping)."""
        p = self.part.cpu().numpy()
        out: dict[int, list[int]] = {}
        for i, x in enumerate(p.tolist()):
            out.setdefault(int(x), []).append(i)
        return out


class InvertedIndexBuilder:
    def __init__(self, store: SplitStore, group=None, device=None, num_reducers: int = 10,
                 capacity: int = 1 << 21, recv_capacity: int = 1 << 21):
        self.store = store
        self.group = group
        self.rank, self.world = D.world_info(group)
        self.device = torch.device(device if device is not None else "cpu")
        self.R = int(num_reducers)
        self.vocab = II.Vocab(self.device, capacity)
        self.rvocab = II.Vocab(self.device, recv_capacity) if self.world > 1 else None
        self.j0, self.j1 = assign_contiguous([store.size(i) for i in range(len(store))], self.rank, self.world)
        self.a, self.b = store.region(self.j0, self.j1)
        lines = store.line_offsets()
        self.line_base = int(lines[self.j0])
        self.rank_lines = int(lines[self.j1] - lines[self.j0])
        self.doc_bits = II.bits_for(self.rank_lines + 1)
        self.text = None
        self.timings: dict[str, float] = {}
        # GPU staging: the rank's text arrives in split-aligned pieces on a copy
        # stream and each piece is mapped as soon as it has landed; two arenas,
        # so build(prefetch_next=True) can start the next build's copies while
        # this one sorts
        cuda = self.device.type == "cuda"
        self.copy_stream = torch.cuda.Stream(self.device) if cuda else None
        self.arenas = [None, None]
        self.slot = 0
        self._prefetched = None  # slot whose copies are in flight
        self.pieces = self._plan_pieces() if cuda else []
        self.events = [[torch.cuda.Event() for _ in self.pieces] for _ in range(2)] if cuda else None
        self.sink = None

    def _plan_pieces(self, first_mb: float = 2, big_mb: float = 24) -> list[tuple[int, int, int]]:
        """Split-aligned pieces (byte start, byte end, line base) of the rank's
        text: a small first piece (its copy is exposed), then ~big_mb ones."""
        offs = self.store.offsets
        lines = self.store.line_offsets()
        out, i = [], self.j0
        target = int(first_mb * (1 << 20))
        while i < self.j1:
            k = i + 1
            while k < self.j1 and offs[k + 1] - offs[i] <= target:
                k += 1
            out.append((int(offs[i] - offs[self.j0]), int(offs[k] - offs[self.j0]), int(lines[i] - lines[self.j0])))
            i = k
            target = int(big_mb * (1 << 20))
        return out

    def _issue_copies(self, slot: int) -> None:
        host = self.store.buffer[self.a:self.b]
        if self.arenas[slot] is None:
            self.arenas[slot] = torch.empty(host.numel(), dtype=torch.uint8, device=self.device)
        dst = self.arenas[slot]
        sp = _hip.stream_ptr(self.copy_stream)
        for (a, b, _), ev in zip(self.pieces, self.events[slot]):
            _hip.call("mr_memcpy_async", _hip.ptr(dst[a:b]), _hip.ptr(host[a:b]), b - a, 1, sp)
            ev.record(self.copy_stream)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def stage(self) -> torch.Tensor:
        """Host -> HBM copy of the rank's splits (pinned buffer, one DMA)."""
        host = self.store.buffer[self.a:self.b]
        if self.device.type == "cuda":
            if self.text is None or self.text.numel() != host.numel():
                self.text = torch.empty(host.numel(), dtype=torch.uint8, device=self.device)
            self.text.copy_(host, non_blocking=True)
        else:
            self.text = host
        return self.text

    def _map_staged(self) -> torch.Tensor:
        """GPU: copies of the rank's pieces (unless prefetched) and one map
        launch per piece once its copy has landed -> posting keys."""
        cur = torch.cuda.current_stream(self.device)
        if self._prefetched != self.slot:
            gate = torch.cuda.Event()
            gate.record(cur)  # the arena may still be read by earlier work
            self.copy_stream.wait_event(gate)
            self._issue_copies(self.slot)
        self._prefetched = None
        text = self.text = self.arenas[self.slot]
        if self.sink is None:
            self.sink = II.PostingSink(self.device, text.numel())
        self.sink.reset()
        for (a, b, lb), ev in zip(self.pieces, self.events[self.slot]):
            cur.wait_event(ev)
            II.map_postings_chunk(text, a, b, lb, self.vocab, self.doc_bits, self.sink)
        return self.sink.finish(self.vocab)

    def build(self, stage: bool = True, prefetch_next: bool = False) -> IndexShard:
        """One inverted-index build of the rank's splits.  ``prefetch_next``:
        start the next build's host->HBM copies (into the other arena) as soon
        as this build's map is done, overlapping them with its sort/shuffle."""
        t0 = time.perf_counter()
        vocab = self.vocab
        vocab.reset()
        if self.device.type == "cuda" and self.b > self.a and (stage or self.text is None):
            keys = self._map_staged()
            text = self.text
            if prefetch_next:
                self._issue_copies(1 - self.slot)
                self._prefetched = 1 - self.slot
        else:
            text = self.stage() if (stage or self.text is None) else self.text
            keys = II.map_postings(text, vocab, self.doc_bits)
        t_map = time.perf_counter()
        bits = vocab.id_bits + self.doc_bits
        if self.world > 1:
            vhi, vlo, vrep = vocab.arrays()
            part, _ = ops.key_meta(vhi, vlo, vrep, text, nparts=self.R, want_len=False)
            dest = (part.to(torch.int64) % self.world).to(torch.int32)
            II.add_dest(keys, dest, self.doc_bits, vocab.id_bits)
            bits += II.bits_for(self.world)
        if bits > 63:
            raise ValueError(f"posting key needs {bits} bits (> 63): lower the table capacity or split the input")
        ukeys = II.sort_unique(keys, bits)
        wid, wstart, docs = II.split_words(ukeys, self.doc_bits, vocab.id_bits, self.line_base)
        vhi, vlo, vrep = vocab.arrays()
        hi, lo, rep = vhi[wid], vlo[wid], vrep[wid]
        t_sort = time.perf_counter()
        if self.world == 1:
            src = text
        else:
            hi, lo, rep, src, wstart, docs = self._shuffle(hi, lo, rep, text, wid, wstart, docs, dest)
        t_shuf = time.perf_counter()
        part, klen = ops.key_meta(hi, lo, rep, src, nparts=self.R)
        koff, kblob = ops.gather_key_bytes(hi, lo, rep, src, lengths=klen)
        self._sync()
        if self._prefetched is not None:
            self.slot = self._prefetched  # the next build maps the prefetched arena
        t1 = time.perf_counter()
        self.timings = {"map": t_map - t0, "sort": t_sort - t_map, "shuffle": t_shuf - t_sort,
                        "finalize": t1 - t_shuf, "total": t1 - t0}
        return IndexShard(hi, lo, koff, kblob, wstart, docs, part)

    # ------------------------------------------------------------------------------
    def _shuffle(self, hi, lo, rep, text, wid, wstart, docs, dest):
        W = self.world
        d = hi.device
        wdest = dest.to(torch.int64)[wid]
        ndocs = wstart[1:] - wstart[:-1]
        _, klen = ops.key_meta(hi, lo, rep, text, want_part=False)
        koff, kblob = ops.gather_key_bytes(hi, lo, rep, text, lengths=klen)
        cnt = torch.zeros(W, 3, dtype=torch.int64, device=d)
        cnt[:, 0].index_add_(0, wdest, torch.ones_like(wdest))
        cnt[:, 1].index_add_(0, wdest, klen.to(torch.int64))
        cnt[:, 2].index_add_(0, wdest, ndocs)
        recv = D.exchange_counts(cnt.view(-1), self.group).view(W, 3)
        both = torch.cat([cnt, recv]).cpu()  # one host sync for all split sizes
        send_c, recv_c = both[:W].tolist(), both[W:].tolist()
        recs = torch.stack([hi, lo, klen.to(torch.int64), ndocs], 1)
        rrecs = D.all_to_all_v(recs, [c[0] for c in send_c], [c[0] for c in recv_c], self.group)
        nbytes = sum(c[1] for c in send_c)
        rblob = D.all_to_all_v(kblob[:nbytes], [c[1] for c in send_c], [c[1] for c in recv_c], self.group)
        rdocs = D.all_to_all_v(docs, [c[2] for c in send_c], [c[2] for c in recv_c], self.group)
        rhi, rlo = rrecs[:, 0].contiguous(), rrecs[:, 1].contiguous()
        rlen, rnd = rrecs[:, 2].contiguous(), rrecs[:, 3].contiguous()
        roff, _ = ops.exclusive_scan(rlen)
        rrep = (roff << REP_LEN_BITS) | rlen
        rv = self.rvocab
        rv.reset()
        rid = II.insert_ids(rv, rhi, rlo, rrep)
        pid = torch.repeat_interleave(rid, rnd, output_size=int(rdocs.numel()))
        rkeys = (pid << 32) | rdocs.to(torch.int64)
        sk = II.sort_unique(rkeys, rv.id_bits + 32)
        wid2, wstart2, docs2 = II.split_words(sk, 32, rv.id_bits, 0)
        vhi, vlo, vrep = rv.arrays()
        return vhi[wid2], vlo[wid2], vrep[wid2], rblob, wstart2, docs2


def naive_index(splits: list[bytes]) -> dict:
    """Oracle: word -> sorted distinct global line ids (SplitStore layout: every
    split followed by a newline unless it already ends in whitespace)."""
    out: dict[bytes, set] = {}
    line = 0
    for s in splits:
        if not (s and s[-1:] in (b"\n", b" ")):
            s = s + b"\n"
        for ln in s.split(b"\n"):
            for w in ln.split():
                out.setdefault(w, set()).add(line)
            line += 1
        line -= 1  # split(b"\n") yields one more piece than there are newlines
    return {k: sorted(v) for k, v in out.items()}
