"""Iterative data-parallel SGD on the digits MLP — the reference's APRIL-ANN
example re-built MI355X-first.

Reference semantics (examples/APRIL-ANN/init.lua, common.lua):
* model "256 inputs 128 tanh 10 log_softmax", multi-class cross-entropy,
  bunch 128, lr 0.01, momentum 0.02, weight decay 1e-4 (not on biases),
  init.lua:6-18,29-55;
* one iteration = 4 map jobs, each the gradient of one random bunch
  (init.lua:65-70,124-141, common.lua:85-104); reduce = sum of gradients and of
  the bunch counts per weight name, loss accumulation (common.lua:112-137);
  finalfn = gradient smoothing by 1/sqrt(N) (common.lua:161-165), optimizer
  step, validation loss, checkpoint, then ``"loop"`` until the stopping rule
  (``max_epochs_wo_imp_relative(2)``, min 20 / max 40 epochs, init.lua:48-54).

MI355X design: the gradient is one fused MFMA forward/backward kernel plus a
deterministic fold, the update one element-wise SGD kernel, both halves of an
epoch replayed as hipGraphs; parameters are ONE flat fp32 vector, and across ranks the
"reduce" phase is ONE RCCL all-reduce of ``[grads | loss, correct, count]``
(SUM) — the shuffle of 4 weight-name partitions degenerates to an all-reduce
because every key goes everywhere.  The server/worker form of the same
workload (map jobs through the coordinator) is
:mod:`lua_mapreduce_1_amd.examples.DigitsMLP`.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import mlp as M
from ..utils import digits

HYPER = dict(bunch_size=128, learning_rate=0.01, momentum=0.02, weight_decay=1e-4, min_epochs=20,
             max_epochs=40, jobs_per_iteration=4, smooth_gradients=True, seed=1234)


@dataclass
class StopRule:
    """``train_holdout_validation{min_epochs, max_epochs,
    stopping_criterion = max_epochs_wo_imp_relative(2)}``: stop once
    epoch >= max_epochs, or epoch >= min_epochs and epoch >= 2 * best_epoch."""
    min_epochs: int = 20
    max_epochs: int = 40
    relative: float = 2.0
    epoch: int = 0
    best_epoch: int = 0
    best_val: float = math.inf
    history: list = field(default_factory=list)

    def update(self, tr_loss: float, va_loss: float) -> bool:
        """Record one epoch; True while training should continue."""
        self.epoch += 1
        self.history.append((self.epoch, tr_loss, va_loss))
        if va_loss < self.best_val:
            self.best_val, self.best_epoch = va_loss, self.epoch
        if self.epoch >= self.max_epochs:
            return False
        return not (self.epoch >= self.min_epochs and self.epoch >= self.relative * max(self.best_epoch, 1))

    def state_string(self) -> str:
        e, tr, va = self.history[-1] if self.history else (0, float("nan"), float("nan"))
        return "%5d %.6f %.6f    %5d %.6f" % (e, tr, va, self.best_epoch, self.best_val)


class DigitsTrainer:
    """Device-resident data + model + optimizer state of one rank."""

    def __init__(self, device="cpu", data=None, hyper: dict | None = None, params: torch.Tensor | None = None):
        self.h = dict(HYPER, **(hyper or {}))
        self.device = torch.device(device)
        tx, ty, vx, vy = data if data is not None else digits.load()
        d = self.device
        self.tx = torch.from_numpy(np.ascontiguousarray(tx)).to(d)
        self.ty = torch.from_numpy(np.ascontiguousarray(ty)).to(d)
        self.vx = torch.from_numpy(np.ascontiguousarray(vx)).to(d)
        self.vy = torch.from_numpy(np.ascontiguousarray(vy)).to(d)
        self.vidx = torch.arange(self.vx.shape[0], dtype=torch.int32, device=d)
        self.w = params.to(d).clone() if params is not None else M.init_params(self.h["seed"], device=d)
        self.v = torch.zeros_like(self.w)
        n = M.LAYOUT.size
        # [grads | loss, correct, count]: the single all-reduce buffer
        self.buf = torch.zeros(n + 3, dtype=torch.float32, device=d)
        self.grads = self.buf[:n]
        self.ws = M.GradWorkspace(self.h["bunch_size"] * self.h["jobs_per_iteration"], d) if d.type == "cuda" else None
        self.vws = M.GradWorkspace(self.vx.shape[0], d) if d.type == "cuda" else None
        self.stop = StopRule(self.h["min_epochs"], self.h["max_epochs"])

    # -- map: gradient of the bunches of some jobs ----------------------------------
    def bunch_indices(self, iteration: int, jobs) -> torch.Tensor:
        """Random pattern indices of map jobs ``jobs`` of ``iteration``
        (reproducible per (seed, iteration, job) so any rank/worker computes
        the same bunch for the same job)."""
        n = self.tx.shape[0]
        out = []
        for j in jobs:
            g = torch.Generator().manual_seed(self.h["seed"] * 1_000_003 + iteration * 1009 + int(j))
            out.append(torch.randint(0, n, (self.h["bunch_size"],), generator=g, dtype=torch.int32))
        idx = torch.cat(out) if out else torch.zeros(0, dtype=torch.int32)
        return idx.to(self.device, non_blocking=True)

    def compute_gradients(self, idx: torch.Tensor) -> None:
        """buf <- [sum_grad | sum_loss, correct, count] of the patterns idx."""
        if idx.numel() == 0:
            self.buf.zero_()
            return
        loss = M.grad_step(self.tx, self.ty, idx, self.w, self.grads, self.ws)
        self.buf[-3:-1].copy_(loss)
        self.buf[-1].fill_(float(idx.numel()))

    # -- final: optimizer step + validation ----------------------------------------
    def apply(self, grads: torch.Tensor, count: float) -> None:
        scale = 1.0 / math.sqrt(max(count, 1.0)) if self.h["smooth_gradients"] else 1.0
        M.sgd_step(self.w, grads, self.v, self.h["learning_rate"], self.h["momentum"], self.h["weight_decay"], scale)

    def validate(self) -> tuple[float, float]:
        loss = M.grad_step(self.vx, self.vy, self.vidx, self.w, None, self.vws, want_grad=False)
        l, ok = loss.tolist()
        n = self.vx.shape[0]
        return l / n, ok / n

    def state(self) -> dict:
        return {"w": self.w.cpu().numpy(), "v": self.v.cpu().numpy()}

    # -- hipGraph-captured epoch -------------------------------------------------
    def capture(self, n_local: int, global_count: int) -> None:
        """Capture the two launch-bound halves of an epoch as hipGraphs (via
        torch.cuda.CUDAGraph, which is hipGraph on ROCm):
          A: fused gradient of the bunch in ``self.static_idx`` -> ``buf``;
          B: SGD update (global bunch count is fixed, so is the smoothing
             scale) + validation forward -> ``self.report``.
        The all-reduce between them stays eager (RCCL), and one 5-float D2H per
        epoch feeds the host-side stopping rule."""
        d = self.device
        self.static_idx = torch.zeros(max(n_local, 1), dtype=torch.int32, device=d)
        self.report = torch.zeros(5, dtype=torch.float32, device=d)
        self.report_host = torch.zeros(5, dtype=torch.float32, pin_memory=True)
        scale = 1.0 / math.sqrt(max(global_count, 1)) if self.h["smooth_gradients"] else 1.0
        h = self.h
        from ..ops import _hip
        _hip.lib()  # load outside capture
        self.graph_a = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_a):
            if n_local:
                loss = M.grad_step(self.tx, self.ty, self.static_idx, self.w, self.grads, self.ws)
                self.buf[-3:-1].copy_(loss)
                self.buf[-1].fill_(float(n_local))
            else:
                self.buf.zero_()
        self.graph_b = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_b):
            M.sgd_step(self.w, self.grads, self.v, h["learning_rate"], h["momentum"], h["weight_decay"], scale)
            vl = M.grad_step(self.vx, self.vy, self.vidx, self.w, None, self.vws, want_grad=False)
            self.report[0:3].copy_(self.buf[-3:])
            self.report[3:5].copy_(vl)


def save_checkpoint(path: str, tr: DigitsTrainer, epoch: int, hist: list, finished: bool) -> None:
    """Trainer snapshot after ``epoch`` (examples/APRIL-ANN/common.lua:191
    serialises the whole trainer to GridFS every iteration): parameters,
    momentum, stopping-rule state and history.  Written atomically."""
    import json
    import os
    st = tr.stop
    meta = {"epoch": epoch, "finished": finished, "hist": hist, "stop": {
        "epoch": st.epoch, "best_epoch": st.best_epoch, "best_val": st.best_val,
        "history": [list(h) for h in st.history]}}
    blob = {"w": tr.w.detach().cpu(), "v": tr.v.detach().cpu(), "meta": json.dumps(meta)}
    tmp = path + ".tmp"
    torch.save(blob, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str) -> dict | None:
    """The snapshot of an unfinished run, or None (missing file, or a finished
    run: common.lua:59-64 resets when ``conf.finished``)."""
    import json
    import os
    if not path or not os.path.exists(path):
        return None
    blob = torch.load(path, weights_only=True)  # tensors + a JSON string: nothing executable
    meta = json.loads(blob["meta"])
    if meta["finished"]:
        return None
    return {"w": blob["w"], "v": blob["v"], **meta}


def train_spmd(device="cpu", group=None, data=None, hyper: dict | None = None, epochs: int | None = None,
               verbose: bool = False, graphs: bool | None = None, checkpoint: str | None = None,
               checkpoint_every: int = 1) -> dict:
    """Iterative DP-SGD, one process per GPU: each rank computes the gradients
    of its share of the iteration's map jobs (one fused launch), one all-reduce
    SUMs ``[grads | loss, correct, count]`` over ranks (RCCL on GPUs), then every
    rank applies the identical optimizer step (replicated parameters, like the
    reference's single finalfn).  On a GPU the two halves of the epoch are
    replayed hipGraphs (``graphs=False`` runs them eagerly).  With
    ``checkpoint`` (a file path) rank 0 snapshots the trainer every
    ``checkpoint_every`` epochs and a relaunch resumes from the snapshot of an
    unfinished run (common.lua:57-77), bit-identical to an uninterrupted run.
    Returns the training history."""
    from ..parallel import dist as D
    import torch.distributed as tdist
    rank, world = D.world_info(group)
    tr = DigitsTrainer(device, data, hyper)
    snap = load_checkpoint(checkpoint) if rank == 0 and checkpoint else None
    if world > 1 and checkpoint:
        snap = D.broadcast_object(snap, 0, group, tr.device if tr.device.type == "cuda" else None)
    hist = []
    it = 0
    if snap is not None:  # before capture: the graphs read w/v in place
        tr.w.copy_(snap["w"])
        tr.v.copy_(snap["v"])
        s = snap["stop"]
        tr.stop.epoch, tr.stop.best_epoch, tr.stop.best_val = s["epoch"], s["best_epoch"], s["best_val"]
        tr.stop.history = [tuple(h) for h in s["history"]]
        hist = list(snap["hist"])
        it = int(snap["epoch"])
    resumed_from = it
    J = tr.h["jobs_per_iteration"]
    jobs = [j for j in range(1, J + 1) if (j - 1) % world == rank]
    B = tr.h["bunch_size"]
    use_graphs = graphs if graphs is not None else tr.device.type == "cuda"
    if use_graphs:
        tr.capture(len(jobs) * B, J * B)
        max_it = epochs if epochs is not None else tr.h["max_epochs"]
        # every epoch's bunch indices, generated once (same streams as eager)
        table = torch.stack([tr.bunch_indices(e, jobs) for e in range(1, max_it + 1)]) if jobs else None
    t0 = time.perf_counter()
    while True:
        it += 1
        if use_graphs:
            if table is not None:
                tr.static_idx.copy_(table[it - 1])
            tr.graph_a.replay()
        else:
            tr.compute_gradients(tr.bunch_indices(it, jobs))
        if world > 1:
            if D._is_gloo(group) and tr.buf.is_cuda:
                h = tr.buf.cpu()
                tdist.all_reduce(h, group=group)
                tr.buf.copy_(h)
            else:
                tdist.all_reduce(tr.buf, group=group)
        if use_graphs:
            tr.graph_b.replay()
            tr.report_host.copy_(tr.report)  # the one synchronising read per epoch
            tot0, tot1, tot2, vl, vok = tr.report_host.tolist()
            tot = [tot0, tot1, tot2]
            nv = tr.vx.shape[0]
            va_loss, va_acc = vl / nv, vok / nv
        else:
            tot = tr.buf[-3:].tolist()
            tr.apply(tr.grads, tot[2])
            va_loss, va_acc = tr.validate()
        tr_loss = tot[0] / max(tot[2], 1.0)
        go = tr.stop.update(tr_loss, va_loss)
        hist.append({"epoch": it, "tr_loss": tr_loss, "va_loss": va_loss, "va_acc": va_acc,
                     "tr_acc": tot[1] / max(tot[2], 1.0)})
        if verbose and rank == 0:
            print(tr.stop.state_string(), flush=True)
        done = (epochs is not None and it >= epochs) or (epochs is None and not go)
        if checkpoint and rank == 0 and (done or it % checkpoint_every == 0):
            save_checkpoint(checkpoint, tr, it, hist, finished=done and epochs is None)
        if done:
            break
    return {"history": hist, "seconds": time.perf_counter() - t0, "params": tr.w, "best_epoch": tr.stop.best_epoch,
            "resumed_from": resumed_from}
