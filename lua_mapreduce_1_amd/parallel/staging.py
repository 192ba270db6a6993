"""Input staging of the SPMD engine (mixed into :class:`~.spmd.SPMDEngine`):
host (pinned) -> HBM copies of a rank's splits on the copy stream, in
growing chunks that the map kernels consume as they land; prefetch of later
iterations' copies into the other arenas; and, for inputs larger than the
HBM arena cap, the streaming rounds through a ring of two arenas.

The reference reads each map job's file from GridFS / disk inside the worker
(/root/reference/mapreduce/utils.lua:133-200, examples/WordCount/mapfn.lua:4);
here the bytes move once per iteration over the GPU's own PCIe link, or
stay resident in HBM across iterations.
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils import trace
from ..utils.config import TUNABLES
from .splits import WindowedSplitStore

N_ARENAS = 3
_PREFETCH_SINGLE = TUNABLES.prefetch_single


class StagingMixin:
    """Copy plans, chunked staging, prefetch and streaming rounds (uses the
    engine's ``arenas``, ``splits``, ``copy_stream``, ``streams`` and
    ``chunk_bytes`` / ``tail_bytes``)."""

    def _plan_chunks(self, ids: list[int], slot: int, single: bool = False):
        """Chunking of a contiguous split range (cached per range): boundaries
        at split boundaries, sizes ramping up (the first copy is exposed), big
        in the middle, ramping down at the end (the last kernel is exposed) —
        also for small per-rank inputs.  Returns (split bounds, arena views,
        pinned host views, reusable events)."""
        a, b = self.splits.region(ids[0], ids[-1] + 1)
        nbytes = b - a
        if self.arenas[slot] is None or self.arenas[slot].numel() < nbytes:
            self.arenas[slot] = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._arena_holds.pop(slot, None)
            self._plans = {k: v for k, v in self._plans.items() if k[2] != slot}

        arena = self.arenas[slot]
        offs = self.splits.offsets
        sizes = []
        rem = nbytes
        up = list(self.chunk_bytes[:-1])
        big = self.chunk_bytes[-1]
        tail = list(self.tail_bytes)
        if single:  # prefetched copies: landed long before the map, one DMA is enough
            up, big, tail = [], max(nbytes, 1), []
        ts = sum(tail)
        while up and rem > up[0] + ts:
            sizes.append(up.pop(0))
            rem -= sizes[-1]
        while rem > big + ts:
            sizes.append(big)
            rem -= big
        if rem > ts:
            sizes.append(rem - ts)
            rem = ts
        for t in tail:
            if rem <= 0:
                break
            sizes.append(min(t, rem))
            rem -= sizes[-1]
        rel = offs[ids[0]:ids[-1] + 2] - offs[ids[0]]
        bidx = np.searchsorted(rel, np.cumsum(sizes), side="left")
        bounds = sorted({0, len(ids)} | {min(int(x), len(ids)) for x in bidx})
        host = self.splits.buffer
        views, host_views, events = [], [], []
        for i in range(len(bounds) - 1):
            ca, cb = self.splits.region(ids[0] + bounds[i], ids[0] + bounds[i + 1])
            views.append(arena[ca - a:cb - a])
            host_views.append(host[ca:cb])
            events.append(torch.cuda.Event() if self.copy_stream is not None else None)
        return bounds, views, host_views, events, ids[0]

    def _get_plan(self, ids: list[int], slot: int, single: bool = False):
        key = (ids[0], len(ids), slot, single)
        plan = self._plans.get(key)
        if plan is None and self.copy_stream is not None and self._can_pipeline() and self.prime_plans and not getattr(
                self, "_priming", False):
            # a pure taskfn maps the same splits every iteration: build (and
            # prime) both copy plans of every arena now, so that no plan is
            # first used — and primed — inside a later, timed iteration
            self._priming = True
            try:
                for sl in range(N_ARENAS):
                    for sg in (False, True):
                        self._get_plan(ids, sl, sg)
            finally:
                self._priming = False
            return self._plans[key]
        if plan is None:
            plan = self._plan_chunks(ids, slot, single)
            self._plans[key] = plan
            if self.copy_stream is not None and self.prime_plans:
                # the first two rounds of a plan's copies behind a cross-stream
                # wait each stalled the host 5-7 ms inside hipMemcpyAsync (a
                # one-time runtime set-up, tools/first_iter.py): take that hit
                # here, once per plan, not in an iteration's copy issue
                for _ in range(2):
                    self._issue_copies(plan, wait_for=torch.cuda.current_stream(self.device))
                    self.copy_stream.synchronize()
        return plan

    def _issue_copies(self, plan, wait_for=None) -> None:
        bounds, views, host_views, events, id0 = plan
        streaming = not self.splits.all_ready()
        cs = self.copy_stream
        if wait_for is not None:
            # the arena may still be read by earlier work (a reused event: a
            # fresh one per iteration grows the runtime's event/signal pool)
            ev0 = self._copy_gate_event()
            ev0.record(wait_for)
            cs.wait_event(ev0)
        from ..ops import _hip
        sp = _hip.stream_ptr(cs)
        for i, (dst, src, ev) in enumerate(zip(views, host_views, events)):
            if streaming:  # the native loader is still reading: copy each chunk once it has landed
                self.splits.wait_ready(id0 + bounds[i], id0 + bounds[i + 1])
            # direct hipMemcpyAsync (pinned -> HBM) instead of copy_: no
            # host-allocator event bookkeeping per chunk (it stalled the host)
            _hip.call("mr_memcpy_async", _hip.ptr(dst), _hip.ptr(src), dst.numel(), 1, sp)
            ev.record(cs)

    def _copy_gate_event(self):
        ev0 = getattr(self, "_copy_gate", None)
        if ev0 is None:
            ev0 = self._copy_gate = torch.cuda.Event()
        return ev0

    def _split_ids(self, jobs, j0, j1):
        ids = [int(v["split"] if isinstance(v, dict) else v) for _, v in jobs[j0:j1]]
        if ids and ids != list(range(ids[0], ids[0] + len(ids))):
            raise ValueError("split jobs of a rank must be contiguous splits")
        return ids

    def _prefetch(self, jobs, j0, j1, q: int) -> None:
        """Start iteration q's host->HBM copies (same splits: the taskfn is
        pure) into its arena now, so the copy engine keeps streaming while
        earlier iterations map, reduce and finalize.  Only for a pure taskfn
        and split inputs; a mismatching plan is re-copied when q runs."""
        if not self._can_pipeline():
            return
        aslot = q % N_ARENAS
        ids = self._split_ids(jobs, j0, j1)
        if not ids or aslot in self._inflight:
            return
        if self.resident and self._arena_holds.get(aslot) == (ids[0], len(ids)):
            return  # HBM-resident input: the arena still holds these splits
        plan = self._get_plan(ids, aslot, single=_PREFETCH_SINGLE)
        # arenas[aslot] was last read by iteration q - N_ARENAS, which has
        # completed (its finalize synchronised): no stream dependency needed
        self._issue_copies(plan)
        self._inflight[aslot] = self._arena_holds[aslot] = (ids[0], len(ids))

    # -- streaming: inputs larger than the HBM arena ----------
    def _arena_cap(self) -> int:
        mb = self.params.get("arena_cap_mb", TUNABLES.arena_cap_mb)
        return int(float(mb) * (1 << 20)) if mb else 0

    def _streaming(self, ids) -> bool:
        cap = self._arena_cap()
        if not cap or not ids:
            return False
        if self.plane_kind not in ("fold", "list", "generic"):
            raise ValueError(f"arena_cap_mb / MR_ARENA_CAP_MB streaming is implemented for the fold, list and "
                             f"general planes (this job runs the {self.plane_kind} plane, which spills with "
                             f"record_cap_mb)")
        a, b = self.splits.region(ids[0], ids[-1] + 1)
        return b - a > cap

    def _stage_streaming(self, jobs, j0, ids):
        """Map a rank's input through a ring of two arena slots of the capped
        size, in rounds of whole splits: round r+1's copies land while round r
        maps; after a round the long keys it introduced move their bytes to a
        persistent key heap at the front of the same buffer (the reference's
        streaming reduce keeps only what it still needs, utils.lua:206-271),
        so the slot can be refilled.  One buffer = one byte source for the
        table's rep words: [key heap | slot 0 | slot 1]."""
        A = self._arena_cap()
        st = self.splits
        sizes = [st.size(i) for i in ids]
        if max(sizes) > A:
            raise ValueError(f"a split of {max(sizes)} bytes does not fit the {A}-byte arena cap")
        rounds, k0, acc = [], 0, 0
        for k, sz in enumerate(sizes):
            if acc + sz > A:
                rounds.append((k0, k))
                k0, acc = k, 0
            acc += sz
        rounds.append((k0, len(ids)))
        a0, b0 = st.region(ids[0], ids[-1] + 1)
        heap_mb = getattr(self, "_stream_heap_mb", TUNABLES.stream_heap_mb)
        H = max(1 << 16, min(b0 - a0, int(heap_mb * (1 << 20))))
        need = H + 2 * A
        buf = getattr(self, "_stream_buf", None)
        if buf is None or buf.numel() < need:
            buf = self._stream_buf = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._stream_heap = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._stream_H = H
        self.arenas[self.slot] = buf
        self._arena_holds.pop(self.slot, None)
        heap = self._stream_heap
        heap.zero_()
        cs = self.copy_stream
        host = st.buffer
        piece = max(self.chunk_bytes[-1], 1)
        plan = []  # per round: [(job range, buffer offset, host offset, bytes)]
        for r, (k0, k1) in enumerate(rounds):
            slot_off = H + (r % 2) * A
            ra = st.region(ids[k0], ids[k0] + 1)[0]
            pieces, k = [], k0
            while k < k1:
                e, acc = k, 0
                while e < k1 and (e == k or acc + sizes[e] <= piece):
                    acc += sizes[e]
                    e += 1
                pa = st.region(ids[k], ids[k] + 1)[0]
                pieces.append(((j0 + k, j0 + e), slot_off + pa - ra, pa, acc, (ids[k], ids[e - 1] + 1)))
                k = e
            plan.append(pieces)
        windowed = isinstance(st, WindowedSplitStore)

        def host_of(r):
            """Host bytes of round r (a window of a windowed store) and the
            host offset of its first byte."""
            k0, k1 = rounds[r]
            if windowed:
                return st.load_round(ids[k0], ids[k1 - 1] + 1, r % 2), st.region(ids[k0], ids[k0] + 1)[0]
            return host, 0

        if cs is None:  # CPU: copy, map, rehome round by round
            for r, pieces in enumerate(plan):
                h, hb = host_of(r)
                for jr, off, ha, n, sp in pieces:
                    st.wait_ready(*sp)
                    buf[off:off + n].copy_(h[ha - hb:ha - hb + n])
                    yield jr, buf[off:off + n]
                self._round_end(buf, H + (r % 2) * A, H + (r % 2) * A + A, heap, H)
            return
        from ..ops import _hip
        cur = torch.cuda.current_stream(self.device)
        evs = getattr(self, "_stream_events", None)
        if evs is None:
            evs = self._stream_events = {"gate": torch.cuda.Event(), "free": [torch.cuda.Event(), torch.cuda.Event()],
                                         "piece": []}
        sp_cs = _hip.stream_ptr(cs)

        def issue(r):
            pe = []
            h, hb = host_of(r)
            for jr, off, ha, n, sp in plan[r]:
                st.wait_ready(*sp)
                _hip.call("mr_memcpy_async", _hip.ptr(buf[off:off + n]), _hip.ptr(h[ha - hb:ha - hb + n]), n, 1,
                          sp_cs)
                ev = torch.cuda.Event()
                ev.record(cs)
                pe.append(ev)
            if windowed:
                st.release(r % 2, pe[-1])  # the window is free once its copies are done
            return pe

        # the buffer may still be read by the previous iteration's tail
        evs["gate"].record(cur)
        cs.wait_event(evs["gate"])
        issued = {0: issue(0)}
        if len(plan) > 1:
            issued[1] = issue(1)
        for r, pieces in enumerate(plan):
            for (jr, off, ha, n, sp), ev in zip(pieces, issued.pop(r)):
                cur.wait_event(ev)
                yield jr, buf[off:off + n]
            self._round_end(buf, H + (r % 2) * A, H + (r % 2) * A + A, heap, H)
            if r + 2 < len(plan):
                evs["free"][r % 2].record(cur)  # slot r % 2 is free once round r's map and rehome ran
                cs.wait_event(evs["free"][r % 2])
                issued[r + 2] = issue(r + 2)

    def _round_end(self, buf, lo: int, hi: int, heap, H: int) -> None:
        """After a streamed round: the fold plane moves the long keys the
        round introduced to the key heap; the list plane also groups the
        round's postings (ListPlane.stream_round_end)."""
        hook = getattr(self.plane, "stream_round_end", None) if self.plane is not None else None
        if hook is not None:
            hook(buf, lo, hi, heap, H)
        else:
            self.table.rehome_long_keys(buf, lo, hi, heap, H)

    def _stage_chunks(self, jobs, j0, j1):
        """Yield (job index range, device tensor) chunks, H2D overlapped with compute."""
        if self.device_input == "split":
            ids = self._split_ids(jobs, j0, j1)
            if not ids:
                return
            if self._streaming(ids):
                yield from self._stage_streaming(jobs, j0, ids)
                return
            cs = self.copy_stream
            key = (ids[0], len(ids))
            prefetched = cs is not None and self._inflight.pop(self.slot, None) == key
            if self.resident and not prefetched and self._arena_holds.get(self.slot) == key:
                # HBM-resident input: these splits were copied into this arena by
                # an earlier, completed iteration — map them in place
                a, b = self.splits.region(ids[0], ids[-1] + 1)
                yield (j0, j0 + len(ids)), self.arena[:b - a]
                return
            plan = self._get_plan(ids, self.slot, single=prefetched and _PREFETCH_SINGLE)
            bounds, views, host_views, events, _ = plan
            if cs is not None and not prefetched and not self.splits.all_ready():
                # input still being read from files (cold start): each chunk is
                # copied as soon as its splits have landed and mapped right
                # behind its copy, so file reads, PCIe and the map overlap
                cur = torch.cuda.current_stream(self.device)
                with trace.range("mr.copies"):
                    gate = self._copy_gate_event()
                    gate.record(cur)
                    cs.wait_event(gate)
                from ..ops import _hip
                sp = _hip.stream_ptr(cs)
                for i in range(len(views)):
                    self.splits.wait_ready(ids[0] + bounds[i], ids[0] + bounds[i + 1])
                    _hip.call("mr_memcpy_async", _hip.ptr(views[i]), _hip.ptr(host_views[i]), views[i].numel(), 1, sp)
                    events[i].record(cs)
                    cur.wait_event(events[i])
                    yield (j0 + bounds[i], j0 + bounds[i + 1]), views[i]
                self._arena_holds[self.slot] = key
                return
            if cs is not None:
                cur = torch.cuda.current_stream(self.device)
                if not prefetched:
                    with trace.range("mr.copies"):
                        self._issue_copies(plan, wait_for=cur)
                    self._arena_holds[self.slot] = key
                # chunks whose copies have already landed (prefetched during the
                # previous iteration's tail) are mapped by ONE launch: a launch's
                # ramp-up and drain cost more than its chunking saves
                done = 0
                while done < len(events) and events[done].query():
                    done += 1
                i0 = 0
                if done >= 2:
                    a0 = views[0].data_ptr() - self.arena.data_ptr()
                    nb = sum(v.numel() for v in views[:done])
                    yield (j0 + bounds[0], j0 + bounds[done]), self.arena[a0:a0 + nb]
                    i0 = done
                for i in range(i0, len(views)):
                    cur.wait_event(events[i])
                    yield (j0 + bounds[i], j0 + bounds[i + 1]), views[i]
            else:
                for i, (dst, src) in enumerate(zip(views, host_views)):
                    self.splits.wait_ready(ids[0] + bounds[i], ids[0] + bounds[i + 1])
                    dst.copy_(src)
                    yield (j0 + bounds[i], j0 + bounds[i + 1]), dst
        elif self.device_input == "file":
            from ..ops import io as mio
            for j in range(j0, j1):
                yield (j, j + 1), mio.load_file(jobs[j][1], self.device)
        else:
            for j in range(j0, j1):
                yield (j, j + 1), jobs[j][1]
