"""Interned, immutable tuples usable as grouping keys.

Reference: /root/reference/mapreduce/tuple.lua — tables emitted as keys or
values are converted into interned immutable tuples (weak 2^18-bucket table,
Jenkins one-at-a-time hash) so that equal contents compare equal and can key
a Lua table.  In Python, ``tuple`` already has value equality and hashing, so
this module keeps the reference's *API* — ``tuple(...)`` converts (nested)
lists into tuples, returns a single scalar unchanged, and interns the result;
``tuple.stats()`` reports live interned tuples — plus the Jenkins OAAT hash
(used by :mod:`..utils` for stable tuple hashing across processes).
"""
from __future__ import annotations

import builtins
import sys
from typing import Any

NUM_BUCKETS = 2 ** 18
_INTERN: dict = {}




builtins_tuple = builtins.tuple


def _convert(v: Any):
    """Nested lists/tuples -> interned tuples, innermost first (tuple.lua:
    230-247 builds nested tuples through the same constructor)."""
    if isinstance(v, (list, builtins_tuple)):
        t = builtins_tuple(_convert(x) for x in v)
        return _INTERN.setdefault(t, t)
    return v


def one_at_a_time(data: bytes, h: int = 0) -> int:
    """Jenkins one-at-a-time hash (tuple.lua:121-140), 32-bit."""
    for c in data:
        h = (h + c) & 0xFFFFFFFF
        h = (h + (h << 10)) & 0xFFFFFFFF
        h ^= h >> 6
    h = (h + (h << 3)) & 0xFFFFFFFF
    h ^= h >> 11
    h = (h + (h << 15)) & 0xFFFFFFFF
    return h


def compute_hash(t) -> int:
    """Deterministic 32-bit hash of a (nested) tuple of numbers/strings."""
    h = 0
    for v in t:
        if isinstance(v, builtins_tuple):
            b = compute_hash(v).to_bytes(4, "little")
        elif isinstance(v, bool):
            b = b"\1" if v else b"\0"
        elif isinstance(v, int):
            b = (v & 0xFFFFFFFF).to_bytes(4, "little")
        elif isinstance(v, bytes):
            b = v
        else:
            b = str(v).encode("utf-8", "surrogateescape")
        for c in b:
            h = (h + c) & 0xFFFFFFFF
            h = (h + (h << 10)) & 0xFFFFFFFF
            h ^= h >> 6
    h = (h + (h << 3)) & 0xFFFFFFFF
    h ^= h >> 11
    h = (h + (h << 15)) & 0xFFFFFFFF
    return h


class _TupleFactory:
    NUM_BUCKETS = NUM_BUCKETS

    def __call__(self, *args):
        if len(args) == 1:
            t = args[0]
            if not isinstance(t, (list, builtins_tuple)):
                return t  # scalars are returned unchanged (tuple.lua:254-256)
        else:
            t = args
        return _convert(t)

    @staticmethod
    def stats():
        """(live tuples, used buckets, load factor) — tuple.lua:332-343.

        Entries referenced only by the intern table are released first (the
        Python analogue of the reference's weak-valued buckets).
        """
        for k in list(_INTERN):
            if sys.getrefcount(k) <= _FREE_REFS:
                del _INTERN[k]
            del k
        n = len(_INTERN)
        buckets = len({compute_hash(k) % NUM_BUCKETS for k in _INTERN}) if n else 1
        return n, buckets, n / NUM_BUCKETS

    @staticmethod
    def is_tuple(x) -> bool:
        return isinstance(x, builtins_tuple)


tuple = _TupleFactory()  # noqa: A001
_FREE_REFS = 5  # dict key + dict value + list + loop variable + call argument


def utest() -> None:
    """tuple.lua:309-328: interning identity, nested tuples, many live
    tuples released once unreferenced, scalars pass through."""
    a = tuple(2, 4, 5, "a", (1, 4, 5))
    b = tuple(2, 4, 5, "a", (1, 4, 5))
    c = tuple([2, 4, 5, "a", [1, 4, 5]])
    assert a is b and a is c
    assert a[4] is tuple(1, 4, 5)
    assert tuple(5) == 5 and tuple("x") == "x"
    base = tuple.stats()[0]
    live = [tuple(i, i + 1) for i in range(10000)]
    assert tuple.stats()[0] >= base + 10000
    del live
    assert tuple.stats()[0] <= base + 1
