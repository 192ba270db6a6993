#!/usr/bin/env python
"""DP-SGD digits MLP (APRIL-ANN analog) step timing: one step = fused MFMA
forward/backward of the iteration's bunches + (N>1) one all-reduce + fused SGD
update + validation forward.  Also times the gradient kernel alone at larger
batches (MFMA throughput check)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lua_mapreduce_1_amd.models import mlp_dpsgd as T  # noqa: E402
from lua_mapreduce_1_amd.ops import mlp as M  # noqa: E402
from lua_mapreduce_1_amd.parallel import dist as D  # noqa: E402


def main() -> int:
    rank, world, device = D.init_from_env()
    T.train_spmd(device, epochs=3)  # warm-up / compile
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = T.train_spmd(device, epochs=40)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"epochs": len(r["history"]), "ms_per_epoch": 1000 * dt / len(r["history"]),
           "final_va_loss": r["history"][-1]["va_loss"], "final_va_acc": r["history"][-1]["va_acc"]}
    tr = T.DigitsTrainer(device)
    for B in (128, 512, 4096, 32768):
        idx = torch.randint(0, tr.tx.shape[0], (B,), dtype=torch.int32, device=device)
        ws = M.GradWorkspace(B, device)
        g = torch.empty(M.LAYOUT.size, device=device)
        M.grad_step(tr.tx, tr.ty, idx, tr.w, g, ws)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            M.grad_step(tr.tx, tr.ty, idx, tr.w, g, ws)
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / 20
        flops = 3 * 2 * B * (256 * 128 + 128 * 10)
        out[f"grad_kernel_B{B}_us"] = us
        out[f"grad_kernel_B{B}_tflops"] = flops / (us * 1e-6) / 1e12
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
