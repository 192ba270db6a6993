"""Checkpoint / resume and fault injection of the SPMD engine (mixed into
:class:`~.spmd.SPMDEngine`).

* the iteration manifest (rank 0): every iteration whose finalfn asked for
  another one, so a relaunched job (torchrun ``--max-restarts``) resumes
  there — the reference keeps its task state in MongoDB and a restarted
  server resumes from it (/root/reference/mapreduce/server.lua:469-502);
* per-rank map checkpoints: a rank's map output of an iteration, so a
  relaunch after a failure later in the iteration re-runs only the maps that
  had not finished (the reference keeps map outputs until the reduce consumes
  them, job.lua:293), with the jobs that ended FAILED / BROKEN;
* ``MR_SPMD_FAULT`` fault injection at the start of an iteration or after its
  map phase.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

from .. import ops
from ..utils import STATUS
from ..utils.config import TUNABLES
from . import dist as D


class CheckpointMixin:
    """Map checkpoints, the iteration manifest and fault injection (uses the
    engine's ``checkpoint_dir``, ``rank``, ``world``, ``iteration`` and
    ``table``)."""

    # -- checkpoint / resume and fault injection -------------------------------
    def _map_ckpt_path(self, iteration: int | None = None) -> str | None:
        """This rank's map output of an iteration (``checkpoint_dir`` only):
        written after the map phase, so a relaunch after a failure later in
        the iteration (shuffle, reduce, another rank's map) re-runs only the
        maps that had not finished — this rank's block of splits is restored
        instead of re-mapped (the reference keeps map outputs
        until the reduce consumes them, job.lua:293, server.lua:475-481)."""
        if not self.checkpoint_dir:
            return None
        import hashlib
        import json
        key = hashlib.sha1(json.dumps(self._manifest_key(), sort_keys=True, default=repr).encode()).hexdigest()[:12]
        it = self.iteration if iteration is None else iteration
        return os.path.join(self.checkpoint_dir, "%s.map.it%d.r%d.w%d.%s" % (self.result_ns, it, self.rank,
                                                                           self.world, key))

    def _save_job_status(self, recs, j0: int, j1: int) -> None:
        """Next to a map checkpoint: the jobs of this rank's block that did
        not end WRITTEN (FAILED / BROKEN, with their repetitions), written
        before the checkpoint itself — a restore then reports the same failed
        maps as the run that wrote it (a failed job stays FAILED,
        server.lua:194-205)."""
        path = self._map_ckpt_path()
        if path is None:
            return
        import json
        bad = {str(j): [int(recs[j].status), int(recs[j].repetitions)] for j in range(j0, j1)
               if recs[j].status in (STATUS.FAILED, STATUS.BROKEN)}
        if not bad:
            if os.path.exists(path + ".jobs.json"):
                os.remove(path + ".jobs.json")  # a stale record of an earlier launch
            return
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        tmp = path + ".jobs.json.tmp"
        with open(tmp, "w") as f:
            json.dump(bad, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path + ".jobs.json")

    def _restore_job_status(self, recs, j0: int, j1: int) -> None:
        """The rank's map jobs after a restore: WRITTEN, except those its
        checkpoint recorded as failed."""
        import json
        now = time.time()
        for j in range(j0, j1):
            recs[j].status, recs[j].started, recs[j].written, recs[j].worker = STATUS.WRITTEN, now, now, self.rank
        path = self._map_ckpt_path()
        if path is None or not os.path.exists(path + ".jobs.json"):
            return
        with open(path + ".jobs.json") as f:
            bad = json.load(f)
        for j, (st, reps) in bad.items():
            j = int(j)
            if j0 <= j < j1:
                recs[j].status, recs[j].repetitions = st, reps

    def _save_map(self, n: int, overflow: bool, recs=None, j0: int = 0, j1: int = 0) -> None:
        path = self._map_ckpt_path()
        if path is None or self.plane_kind != "fold" or overflow:
            return
        if recs is not None:
            self._save_job_status(recs, j0, j1)
        from ..runtime import codec
        hi, lo, val, rep = self.table.compact((n, False))
        _, ln = ops.key_meta(hi, lo, rep, self._source(), want_part=False)
        off, blob = ops.gather_key_bytes(hi, lo, rep, self._source(), lengths=ln)
        h = lambda t: t.detach().cpu().numpy()  # noqa: E731
        data = codec.encode_columnar(h(hi).view(np.uint64), h(lo).view(np.uint64), h(val), h(off), h(blob))
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    def _restore_map(self, jobs, recs, j0: int, j1: int) -> bool:
        """Load this rank's map output of the current iteration from its
        checkpoint, if an earlier launch wrote it: the table is refilled from
        the saved keys (their bytes become the tail's key source) and the
        rank's map jobs are WRITTEN without running."""
        path = self._map_ckpt_path()
        if path is None or self.plane_kind != "fold" or not os.path.exists(path):
            return False
        from ..runtime import codec
        with open(path, "rb") as f:
            cols = codec.decode_columnar(f.read())
        d = self.device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(d)  # noqa: E731
        koff = cols["key_off"].astype(np.int64)
        lens = np.diff(koff).astype(np.uint64)
        rep = t(((koff[:-1].astype(np.uint64)) << np.uint64(24)) | lens)
        blob = torch.from_numpy(np.concatenate([cols["key_blob"], np.zeros(1, np.uint8)])).to(d)
        self._restored_src = blob
        n = int(cols["hi"].size)
        if 2 * n > self.table.cap:
            self.table = ops.HashTable(ops.next_pow2(4 * n), device=d, op=self.op)
            self._table_capacity = self.table.cap
        timer = self._timer()
        if timer is not None:
            timer.begin()
        self.table.insert(t(cols["hi"]), t(cols["lo"]), t(cols["val"]), rep, src=blob)
        self.maps_restored += 1
        self._restore_job_status(recs, j0, j1)
        self._chunks[self.tslot] = []
        self._log("# rank %d: map of iteration %d restored from %s\n" % (self.rank, self.iteration, path))
        sys.stderr.write("# rank %d: map of iteration %d restored from its checkpoint\n" % (self.rank, self.iteration))
        return True

    def _drop_map_ckpt(self, iteration: int) -> None:
        path = self._map_ckpt_path(iteration)
        for p in (path, path + ".jobs.json") if path is not None else ():
            if os.path.exists(p):
                os.remove(p)

    def _manifest_path(self) -> str | None:
        if not self.checkpoint_dir:
            return None
        return os.path.join(self.checkpoint_dir, "%s.spmd.json" % self.result_ns)

    def _manifest_key(self) -> dict:
        """Identity of the job a manifest belongs to: a relaunch with other
        modules, partition count or init args starts from scratch."""
        import hashlib
        import json
        p = self.params
        try:
            args = json.dumps(p.get("init_args"), sort_keys=True, default=repr)
        except (TypeError, ValueError):
            args = repr(p.get("init_args"))
        return {k: p.get(k) for k in ("taskfn", "mapfn", "partitionfn", "reducefn", "finalfn", "combinerfn",
                                      "num_partitions")} | {
            "world": self.world, "init_args": hashlib.sha1(args.encode()).hexdigest()}

    def _load_manifest(self) -> int:
        """Iterations already finished by an earlier launch of this same task
        (server.lua:469-502 restart semantics: an unfinished task resumes, a
        FINISHED one starts again from scratch).  Rank 0 decides, all agree."""
        start = 0
        path = self._manifest_path()
        if self.rank == 0 and path and os.path.exists(path):
            import json
            with open(path) as f:
                m = json.load(f)
            if m.get("key") == self._manifest_key() and not m.get("finished"):
                start = int(m.get("iteration", 0))
        if self.world > 1:
            start = D.broadcast_object(start, 0, self.group, self.device if self.device.type == "cuda" else None)
        return start

    def _save_manifest(self, finished: bool) -> None:
        path = self._manifest_path()
        if self.rank != 0 or not path:
            return
        import json
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"key": self._manifest_key(), "iteration": self.iteration, "finished": finished,
                       "time": time.time()}, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)  # atomic: a crash leaves the old or the new manifest

    def _maybe_inject_fault(self, phase: str = "start") -> None:
        """``MR_SPMD_FAULT=<iteration>:<rank>:raise|exit[:<attempt>[:<phase>]]``
        (SURVEY.md §5.3): that rank fails in that iteration — at its start
        (phase ``start``, the default) or after the map phase (``shuffle``:
        every rank's map output of the iteration is already checkpointed) —
        ``exit`` leaves its peers blocked in a collective, as a lost GPU or
        node would."""
        spec = os.environ.get("MR_SPMD_FAULT", TUNABLES.spmd_fault)
        if not spec:
            return
        f = spec.split(":")
        it, rk, action = f[:3]
        want_phase = f[4] if len(f) > 4 and f[4] else "start"
        cur = self.iteration + 1 if phase == "start" else self.iteration
        if want_phase != phase or int(it) != cur or int(rk) != self.rank:
            return
        # optional 4th field: only in that torchrun attempt (0 = first launch; empty = any)
        if len(f) > 3 and f[3] != "" and int(f[3]) != int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")):
            return
        if action == "exit":
            sys.stderr.write("# injected fault: rank %d exits at iteration %d (%s)\n" % (self.rank, cur, phase))
            sys.stderr.flush()
            os._exit(17)
        raise RuntimeError("injected fault: rank %d at iteration %d (%s)" % (self.rank, cur, phase))
