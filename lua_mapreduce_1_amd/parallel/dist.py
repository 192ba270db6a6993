"""Process-group plumbing and the shuffle collectives.

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL on
ROCm, over xGMI inside a node) for device tensors, ``gloo`` for CPU runs and
tests.  The MapReduce shuffle (GridFS / scp / shared FS
in the reference) is an all-to-all-v in two steps: the int64 per-destination
counts first, then the payload, each a single ``all_to_all_single`` so every
xGMI link is driven concurrently (an all-to-all is bounded by per-link
bandwidth x 7 links, not by a ring).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..utils.config import TUNABLES


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init_from_env(backend: str | None = None, timeout_s: float | None = None, use_gpu: bool | None = None):
    """Initialise the default group from torchrun's env (no-op for WORLD_SIZE=1).

    ``timeout_s`` (default ``MR_COLL_TIMEOUT``) bounds every collective: a
    rank that hangs or dies makes its peers' collectives fail after it instead
    of blocking forever (SURVEY.md §5.3 failure detection), and torchrun's
    ``--max-restarts`` then relaunches the job.

    Returns (rank, world, device)."""
    if timeout_s is None:
        timeout_s = TUNABLES.coll_timeout
    rank, world, local = env_world()
    if use_gpu is None:
        use_gpu = torch.cuda.is_available() and backend != "gloo"
    if use_gpu:
        ndev = torch.cuda.device_count()
        local = local % max(ndev, 1)  # several ranks may share a GPU (gloo tests)
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
        from ..utils import numa
        numa.bind_to_gpu(device.index or 0)  # pinned buffers allocated later land on the GPU's socket
    if world > 1 and not dist.is_initialized():
        # more ranks than GPUs (a rehearsal on a 1-GPU box): RCCL refuses two
        # ranks on one device, so such a job runs its collectives over gloo
        be = backend or ("nccl" if use_gpu and world <= torch.cuda.device_count() else "gloo")
        kw = {}
        if be == "nccl" and use_gpu:
            kw["device_id"] = device
        td = datetime.timedelta(seconds=timeout_s)
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        if attempt != "0" and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
            # a torchrun relaunch (--max-restarts) talks to the same agent-hosted
            # store as the failed attempt, whose peer addresses are still in it:
            # key this attempt's rendezvous apart
            store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                  is_master=False, timeout=td)
            kw["store"] = dist.PrefixStore("mr_attempt_%s" % attempt, store)
        dist.init_process_group(be, rank=rank, world_size=world, timeout=td, **kw)
    return rank, world, device


def initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_info(group=None) -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _is_gloo(group=None) -> bool:
    return dist.get_backend(group) == "gloo"


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    if not _is_gloo(group):
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
        return
    # gloo (CPU tests, or several ranks sharing one GPU): collectives run on
    # host copies; point-to-point fallback when all_to_all is unavailable.
    dev = inp.device
    ci, co = inp.cpu(), torch.empty(out.shape, dtype=out.dtype)
    try:
        dist.all_to_all_single(co, ci, out_splits, in_splits, group=group)
    except RuntimeError:
        rank, world = world_info(group)
        n_in = in_splits or [ci.shape[0] // world] * world
        n_out = out_splits or [co.shape[0] // world] * world
        ins = list(torch.split(ci, n_in))
        outs = list(torch.split(co, n_out))
        reqs = []
        for p in range(world):
            if p == rank:
                outs[p].copy_(ins[p])
                continue
            reqs.append(dist.isend(ins[p].contiguous(), p, group=group))
            reqs.append(dist.irecv(outs[p], p, group=group))
        for r in reqs:
            r.wait()
    out.copy_(co.to(dev) if dev.type != "cpu" else co)


def exchange_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    """counts[p] = items this rank sends to p -> recv[p] = items p sends here."""
    recv = torch.empty_like(counts)
    _a2a(recv, counts, None, None, group)
    return recv


def all_to_all_v(payload: torch.Tensor, send_counts: list[int], recv_counts: list[int], group=None) -> torch.Tensor:
    """Variable all-to-all along dim 0 (rows of any trailing shape)."""
    shape = (sum(recv_counts),) + tuple(payload.shape[1:])
    out = torch.empty(shape, dtype=payload.dtype, device=payload.device)
    _a2a(out, payload.contiguous(), list(recv_counts), list(send_counts), group)
    return out


def all_to_all_v_into(out: torch.Tensor, payload: torch.Tensor, send_counts: list[int], recv_counts: list[int],
                      group=None, async_op: bool = False):
    """all_to_all_v into a caller's buffer ``out`` (rows of ``sum(recv_counts)``).
    ``async_op`` (RCCL): returns the work handle right away — the exchange
    runs on the collective's own stream while the caller queues more work on
    its stream; ``wait()`` before reading ``out`` (gloo: done on return, None)."""
    if async_op and not _is_gloo(group):
        return dist.all_to_all_single(out, payload.contiguous(), list(recv_counts), list(send_counts), group=group,
                                      async_op=True)
    _a2a(out, payload.contiguous(), list(recv_counts), list(send_counts), group)
    return None


def all_to_all_bytes(payloads: list, device=None, group=None) -> list:
    """payloads[d] (bytes) goes to rank d; returns the byte strings every rank
    sent here, in rank order.  Two collectives whatever the world size: the
    int64 byte counts, then ONE uint8 all_to_all_single of the concatenated
    payloads (on the device for RCCL, on the host for gloo).  Every payload
    carries one pad byte, so no rank sends or receives an empty tensor."""
    rank, world = world_info(group)
    dev = _coll_device(torch.device(device) if device is not None else torch.device("cpu"), group)
    send = [len(b) + 1 for b in payloads]
    counts = torch.tensor(send, dtype=torch.int64)
    recv = exchange_counts(counts.to(dev), group).cpu().tolist()
    blob = b"".join(b + b"\0" for b in payloads)
    buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    out = all_to_all_v(buf, send, recv, group).cpu().numpy().tobytes()
    res, o = [], 0
    for n in recv:
        res.append(out[o:o + n - 1])
        o += n
    return res


def barrier(group=None, device=None) -> None:
    if dist.is_available() and dist.is_initialized():
        if device is not None and torch.device(device).type == "cuda" and not _is_gloo(group):
            dist.barrier(group=group, device_ids=[torch.device(device).index])
        else:
            dist.barrier(group=group)


def _coll_device(device, group=None):
    return torch.device("cpu") if _is_gloo(group) else device


def all_reduce_max(x: float, device, group=None) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device(device, group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_reduce_sum_int(x: int, device, group=None) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.int64, device=_coll_device(device, group))
    dist.all_reduce(t, group=group)
    return int(t.item())


def broadcast_object(obj, src: int = 0, group=None, device=None):
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group, device=None if _is_gloo(group) else device)
    return lst[0]


def gather_objects(obj, dst: int = 0, group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    rank, world = world_info(group)
    out = [None] * world if rank == dst else None
    dist.gather_object(obj, out, dst=dst, group=group)
    return out


def all_gather_object(obj, group=None) -> list:
    """Every rank's ``obj`` (in rank order) on every rank."""
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    _, world = world_info(group)
    out = [None] * world
    dist.all_gather_object(out, obj, group=group)
    return out


def all_gather_tensor(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenation of every rank's equally-shaped ``t`` along dim 0."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    _, world = world_info(group)
    if _is_gloo(group):
        h = t.cpu().contiguous()
        out = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(out, h, group=group)
        return torch.cat(out).to(t.device)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out
