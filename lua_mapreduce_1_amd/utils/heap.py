"""Binary min-heap with a custom "less than" comparator.

Reference: /root/reference/mapreduce/heap.lua:20-120 (top/pop/push/clear/size/
empty, ctor ``heap(cmp)``).  Used by :func:`..utils.merge_iterator` for the
host-side k-way merge of sorted intermediate runs (the device path re-sorts
with the radix kernels instead).
"""
from __future__ import annotations

from typing import Any, Callable, Optional


class heap:  # noqa: N801  (mirrors the reference's lowercase class name)
    __slots__ = ("data", "cmp")

    def __init__(self, cmp: Optional[Callable[[Any, Any], bool]] = None):
        self.cmp = cmp or (lambda a, b: a < b)
        self.data: list = []

    def top(self):
        return self.data[0] if self.data else None

    def pop(self) -> None:
        data, cmp = self.data, self.cmp
        if not data:
            return
        v = data.pop()
        n = len(data)
        if n == 0:
            return
        pos = 0
        while True:
            left = 2 * pos + 1
            if left >= n:
                break
            right = left + 1
            child = right if (right < n and cmp(data[right], data[left])) else left
            if cmp(data[child], v):
                data[pos] = data[child]
                pos = child
            else:
                break
        data[pos] = v

    def push(self, v) -> None:
        data, cmp = self.data, self.cmp
        data.append(v)
        pos = len(data) - 1
        while pos > 0:
            p = (pos - 1) // 2
            if cmp(v, data[p]):
                data[pos] = data[p]
                pos = p
            else:
                break
        data[pos] = v

    def clear(self) -> None:
        self.data = []

    def size(self) -> int:
        return len(self.data)

    def empty(self) -> bool:
        return not self.data

    def __len__(self) -> int:
        return len(self.data)


def utest() -> None:
    """heap.lua:99-118: pop order against a sort."""
    import random
    rng = random.Random(1234)
    data = [rng.random() for _ in range(1000)]
    h = heap()
    for x in data:
        h.push(x)
    out = []
    while not h.empty():
        out.append(h.top())
        h.pop()
    assert out == sorted(data)
    h2 = heap(lambda a, b: a > b)
    for x in data:
        h2.push(x)
    assert h2.size() == len(data) and h2.top() == max(data)
    h2.clear()
    assert h2.empty()
