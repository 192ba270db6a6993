"""Fused MLP gradient step + SGD update (HIP, gfx950 MFMA) for the iterative
DP-SGD workload — the APRIL-ANN example of the reference
(/root/reference/mapreduce/examples/APRIL-ANN/init.lua:10-12 "256 inputs 128
tanh 10 log_softmax", bunch 128; gradients common.lua:85-104, reduction
common.lua:112-137, optimizer step common.lua:144-202).

Parameters live in ONE flat fp32 vector ``[W1 (IN*HID) | b1 | W2 (HID*OUT) | b2]``
so the gradient all-reduce is a single collective and the optimizer one
element-wise launch.  ``W1[i, j]`` is input i -> hidden j (row-major).

``grad_step`` is one kernel launch on a GPU (csrc/hip/mlp.hip); on CPU tensors it
runs the same math in PyTorch fp32 (the non-GPU path; also the numerics
reference of the tests).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

IN, HID, OUT = 256, 128, 10
ROWS_PER_BLOCK = 16


@dataclass(frozen=True)
class Layout:
    inp: int = IN
    hid: int = HID
    out: int = OUT

    @property
    def w1(self):
        return slice(0, self.inp * self.hid)

    @property
    def b1(self):
        o = self.inp * self.hid
        return slice(o, o + self.hid)

    @property
    def w2(self):
        o = self.inp * self.hid + self.hid
        return slice(o, o + self.hid * self.out)

    @property
    def b2(self):
        o = self.inp * self.hid + self.hid + self.hid * self.out
        return slice(o, o + self.out)

    @property
    def size(self) -> int:
        return self.inp * self.hid + self.hid + self.hid * self.out + self.out

    def views(self, flat: torch.Tensor) -> dict:
        return {"w1": flat[self.w1].view(self.inp, self.hid), "b1": flat[self.b1],
                "w2": flat[self.w2].view(self.hid, self.out), "b2": flat[self.b2]}


LAYOUT = Layout()
WEIGHT_NAMES = ("w1", "b1", "w2", "b2")


def init_params(seed: int = 1234, inf: float = -1.0, sup: float = 1.0, device="cpu",
                layout: Layout = LAYOUT) -> torch.Tensor:
    """Uniform [inf, sup] / sqrt(fan_in) per layer, biases included (the
    reference's ``randomize_weights{inf=-1, sup=1, use_fanin=true}``,
    init.lua:39-44; exact APRIL-ANN RNG stream not reproduced)."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.empty(layout.size, dtype=torch.float32)
    for sl, fan in ((layout.w1, layout.inp), (layout.b1, layout.inp), (layout.w2, layout.hid),
                    (layout.b2, layout.hid)):
        n = sl.stop - sl.start
        flat[sl] = (torch.rand(n, generator=g) * (sup - inf) + inf) / math.sqrt(fan)
    return flat.to(device)


class GradWorkspace:
    """Per-device scratch of the fused kernel: block partials and the
    last-block counter (kept zeroed by the kernel itself)."""

    def __init__(self, max_batch: int, device, layout: Layout = LAYOUT):
        nb = (max_batch + ROWS_PER_BLOCK - 1) // ROWS_PER_BLOCK
        self.max_batch = max_batch
        self.partials = torch.empty(nb * (layout.size + 2), dtype=torch.float32, device=device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=device)
        self.loss = torch.zeros(2, dtype=torch.float32, device=device)


def reference_forward_backward(X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor, params: torch.Tensor,
                               layout: Layout = LAYOUT, want_grad: bool = True):
    """Plain PyTorch fp32 autograd version (the numerics reference)."""
    p = params.detach().clone().requires_grad_(want_grad)
    v = layout.views(p)
    x = X[idx.long()]
    y = labels[idx.long()].long()
    h = torch.tanh(x @ v["w1"] + v["b1"])
    z = h @ v["w2"] + v["b2"]
    logp = torch.log_softmax(z, dim=1)
    losses = -logp.gather(1, y[:, None])[:, 0]
    loss = losses.sum()
    correct = (z.argmax(1) == y).sum().float()
    grads = None
    if want_grad:
        loss.backward()
        grads = p.grad.detach()
    return grads, torch.stack([loss.detach(), correct])


def grad_step(X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor, params: torch.Tensor,
              grads: torch.Tensor | None, ws: GradWorkspace | None = None, want_grad: bool = True,
              layout: Layout = LAYOUT) -> torch.Tensor:
    """Summed-loss gradient of the bunch ``idx`` into ``grads`` (flat, fp32);
    returns a 2-vector [sum of losses, correct predictions] (device tensor)."""
    B = int(idx.numel())
    if X.is_cuda:
        from . import _hip as H
        if ws is None or ws.max_batch < B:
            ws = GradWorkspace(B, X.device, layout)
        g = grads if want_grad else ws.partials  # unused when want_grad = 0
        H.call("mr_mlp_grad", H.ptr(X), H.ptr(labels), H.ptr(idx), B, layout.inp, layout.hid, layout.out,
               H.ptr(params), H.ptr(g), H.ptr(ws.loss), H.ptr(ws.partials), H.ptr(ws.counter),
               1 if want_grad else 0, H.stream(X.device))
        return ws.loss
    gr, loss = reference_forward_backward(X, labels, idx, params, layout, want_grad)
    if want_grad:
        grads.copy_(gr)
    return loss


def sgd_step(w: torch.Tensor, g: torch.Tensor, v: torch.Tensor, lr: float, momentum: float, weight_decay: float,
             scale: float = 1.0, layout: Layout = LAYOUT) -> None:
    """v <- momentum*v - lr*(scale*g + wd*w [weights only]);  w <- w + v."""
    if w.is_cuda:
        from . import _hip as H
        H.call("mr_mlp_sgd", H.ptr(w), H.ptr(g), H.ptr(v), int(w.numel()), float(lr), float(momentum),
               float(weight_decay), float(scale), layout.b1.start, layout.b1.stop, layout.b2.start,
               H.stream(w.device))
        return
    decay = torch.full_like(w, weight_decay)
    decay[layout.b1] = 0
    decay[layout.b2] = 0
    d = scale * g + decay * w
    v.mul_(momentum).sub_(lr * d)
    w.add_(v)
