"""Input staging: files / byte strings -> (pinned) host -> device tensors."""
from __future__ import annotations

import os

import torch


def read_file_bytes(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def bytes_to_device(data: bytes, device=None, pin: bool = True) -> torch.Tensor:
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.zeros(0, dtype=torch.uint8)
    if device is None or torch.device(device).type == "cpu":
        return t
    if pin:
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


def load_file(path: str, device=None) -> torch.Tensor:
    """Whole file as a uint8 tensor on ``device`` (host tensor when None/cpu)."""
    n = os.path.getsize(path)
    if device is None or torch.device(device).type == "cpu":
        t = torch.empty(n, dtype=torch.uint8)
        with open(path, "rb") as f:
            f.readinto(memoryview(t.numpy()))
        return t
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    with open(path, "rb") as f:
        f.readinto(memoryview(host.numpy()))
    return host.to(device, non_blocking=True)
