"""Bind a rank's CPU threads to the NUMA node of its GPU.

One process per GPU stages its input from pinned host memory every
iteration (the PCIe link is the bound of a host-staged step).  On a
two-socket MI355X node each socket hosts four of the eight GPUs; a rank whose
pinned buffers sit on the other socket's memory pulls every staged byte
through the socket-to-socket link, shared with the other ranks doing the
same.  Pinned pages are placed where they are first touched, so restricting
the rank's threads (the split loader's threads are created later and inherit
the mask) to the CPUs of the GPU's node before any buffer is allocated keeps
the staging traffic on the local socket.  This replaces nothing in the
reference (its workers are CPU processes reading GridFS); it is the HBM-side
counterpart of `numactl --cpunodebind` for the SPMD ranks.

The GPU's node comes from sysfs (``/sys/bus/pci/devices/<bdf>/numa_node``)
through its PCI address; the CPUs from ``/sys/devices/system/node/node<N>/
cpulist``, intersected with the CPUs the process may already use (cgroup
cpusets).  Anything missing or unreadable leaves the affinity unchanged.
"""
from __future__ import annotations

import os

SYS = "/sys"


def parse_cpulist(text: str) -> set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    out: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def gpu_pci_address(device_index: int) -> str | None:
    """'dddd:bb:dd.0' of a visible GPU (torch's device properties), or None."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        bus = getattr(p, "pci_bus_id", None)
        dev = getattr(p, "pci_device_id", None)
        dom = getattr(p, "pci_domain_id", 0) or 0
        if bus is None or dev is None:
            return None
        return f"{int(dom):04x}:{int(bus):02x}:{int(dev):02x}.0"
    except Exception:  # noqa: BLE001 - no GPU / older torch: leave the affinity alone
        return None


def numa_node_of(pci: str, sys_root: str = SYS) -> int | None:
    try:
        with open(os.path.join(sys_root, "bus", "pci", "devices", pci, "numa_node")) as f:
            n = int(f.read().strip())
        return n if n >= 0 else None
    except (OSError, ValueError):
        return None


def node_cpus(node: int, sys_root: str = SYS) -> set[int]:
    try:
        with open(os.path.join(sys_root, "devices", "system", "node", f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return set()


def bind_cpus_to_node(node: int | None, sys_root: str = SYS) -> set[int] | None:
    """Restrict this process to the allowed CPUs of ``node``; returns the new
    mask, or None when nothing was changed."""
    if node is None or not hasattr(os, "sched_setaffinity"):
        return None
    cpus = node_cpus(node, sys_root) & set(os.sched_getaffinity(0))
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return cpus


def bind_to_gpu(device_index: int, sys_root: str = SYS) -> dict:
    """Bind this rank to its GPU's NUMA node (MR_NUMA_BIND=0 turns it off).
    Returns {"pci", "node", "cpus"} for the log (cpus: count bound, 0 if not)."""
    from .config import TUNABLES
    info = {"pci": None, "node": None, "cpus": 0}
    if not TUNABLES.numa_bind:
        return info
    pci = gpu_pci_address(device_index)
    info["pci"] = pci
    if pci is None:
        return info
    node = numa_node_of(pci, sys_root)
    info["node"] = node
    cpus = bind_cpus_to_node(node, sys_root)
    info["cpus"] = len(cpus) if cpus else 0
    return info
