"""Interned, immutable tuples usable as grouping keys.

Reference: /root/reference/mapreduce/tuple.lua — tables emitted as keys or
values are converted into interned immutable tuples (weak 2^18-bucket table,
Jenkins one-at-a-time hash) so that equal contents compare equal and can key
a Lua table.  In Python, ``tuple`` already has value equality and hashing, so
this module keeps the reference's *API* — ``tuple(...)`` converts (nested)
lists into tuples, returns a single scalar unchanged, and interns the result;
``tuple.stats()`` reports live interned tuples — plus the Jenkins OAAT hash
(used by :mod:`..utils` for stable tuple hashing across processes).

Interning mimics the reference's weak-valued buckets (tuple.lua:250-302): a
CPython tuple cannot be weakly referenced, so the intern table is pruned of
entries nobody else references whenever it has doubled since the last prune
(amortised O(1) per insert) — a long-running worker that emits millions of
distinct list keys keeps only the live ones.
"""
from __future__ import annotations

import builtins
import sys
from typing import Any

NUM_BUCKETS = 2 ** 18
PRUNE_MIN = 1 << 16  # entries before the first prune

builtins_tuple = builtins.tuple
_INTERN: dict = {}
_limit = PRUNE_MIN


def _calibrate_dead_refs() -> int:
    """getrefcount of an entry nobody else references, measured in the same
    comprehension shape _prune uses (the count includes the table's key and
    value, the loop variable and the call's argument on CPython 3.10, but
    interpreters differ: 3.14 borrows stack references and reports less)."""
    probe: dict = {}
    t = builtins_tuple([object()])
    probe[t] = t
    del t
    return [sys.getrefcount(k) for k in probe][0]


_DEAD_REFS = _calibrate_dead_refs()


def _prune() -> None:
    """Drop entries referenced only by the table (reference count at most
    the calibrated one of an unreferenced entry).  Outer tuples go first, so
    a pass repeats while it frees anything."""
    global _limit
    while True:
        dead = [k for k in _INTERN if sys.getrefcount(k) <= _DEAD_REFS]
        for k in dead:
            del _INTERN[k]
        n = len(dead)
        del dead
        if not n:
            break
    _limit = max(PRUNE_MIN, 2 * len(_INTERN))


def _convert(v: Any):
    """Nested lists/tuples -> interned tuples, innermost first (tuple.lua:
    230-247 builds nested tuples through the same constructor)."""
    if isinstance(v, (list, builtins_tuple)):
        t = builtins_tuple(_convert(x) for x in v)
        r = _INTERN.setdefault(t, t)
        if r is t and len(_INTERN) > _limit:
            _prune()
        return r
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
        """(live tuples, used buckets, load factor) — tuple.lua:332-343
        (unreferenced entries are released first)."""
        _prune()
        n = len(_INTERN)
        buckets = len({compute_hash(k) % NUM_BUCKETS for k in _INTERN}) if n else 1
        return n, buckets, n / NUM_BUCKETS

    @staticmethod
    def is_tuple(x) -> bool:
        return isinstance(x, builtins_tuple)


tuple = _TupleFactory()  # noqa: A001


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
    # an interned tuple held across a forced prune keeps its identity
    held = tuple(["held", 1, [2, 3]])
    _prune()
    assert tuple(["held", 1, [2, 3]]) is held and held[2] is tuple(2, 3)
