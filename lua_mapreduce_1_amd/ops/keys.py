"""Host (NumPy) definition of the 128-bit key encoding used by the device ops.

This module is the executable specification of ``csrc/hip/mr_common.h`` and
the CPU implementation of the device primitives for CPU tensors / tests.

Key of a byte string ``b`` (the replacement for the reference's interned
Lua strings/tuples, /root/reference/mapreduce/tuple.lua:121-140):

* ``len(b) <= 15``: exact — ``hi`` = b[0:8] big-endian, ``lo`` = b[8:15]
  big-endian ``<< 8 | len``; unsigned (hi, lo) order == bytewise order (the
  order Lua string ``<`` gives, utils.lua:126).
* ``len(b) >= 16``: ``hi`` = b[0:8] big-endian (exact prefix),
  ``lo`` = 56-bit hash ``<< 8 | 0xFF``.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
PACK_MAX = 15
LONG_MARK = 0xFF
REP_LEN_BITS = 24
REP_LEN_MASK = (1 << REP_LEN_BITS) - 1
FNV_PRIME = 16777619
FNV_OFFSET = 2166136261
WS = b" \t\n\v\f\r"  # Lua %s in the C locale (examples/WordCount/mapfn.lua:5)

_WS_TABLE = np.zeros(256, dtype=bool)
for _c in WS:
    _WS_TABLE[_c] = True


def fmix64(x: int) -> int:
    x &= M64
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


def long_hash(b: bytes) -> int:
    n = len(b)
    h = 0x243F6A8885A308D3 ^ ((n * 0x13198A2E03707344) & M64)
    for w in range(0, n, 8):
        word = int.from_bytes(b[w:w + 8], "little")
        h = (fmix64(h ^ word) * 0x9E3779B97F4A7C15) & M64
    return h


# Debug knob: only the low bits of the 56-bit long-key hash are kept, so
# distinct long keys collide (tests of the exact byte verification).  Host and
# device must agree: set it with :func:`set_long_hash_bits`.
LONG_HASH_MASK = M64


def set_long_hash_bits(bits: int | None) -> None:
    """Keep ``bits`` bits of the long-key hash (None: all of them) on the host
    and in every loaded kernel translation unit."""
    global LONG_HASH_MASK
    LONG_HASH_MASK = M64 if bits is None else (1 << int(bits)) - 1
    import torch
    if torch.cuda.is_available():
        from . import _hip
        _hip.set_long_mask(LONG_HASH_MASK)


def long_lo(h: int) -> int:
    return (((fmix64(h) & LONG_HASH_MASK) << 8) & M64) | LONG_MARK


def pack_key(b: bytes) -> tuple[int, int]:
    """(hi, lo) of a byte string."""
    n = len(b)
    if n == 0:
        raise ValueError("empty key")
    hi = int.from_bytes(b[:8].ljust(8, b"\0"), "big")
    if n <= PACK_MAX:
        lo = (int.from_bytes(b[8:15].ljust(7, b"\0"), "big") << 8) | n
    else:
        lo = long_lo(long_hash(b))
    return hi, lo


def is_long(lo) -> bool:
    return (int(lo) & 0xFF) == LONG_MARK


def unpack_key(hi: int, lo: int) -> bytes:
    """Bytes of a packed (short) key."""
    hi &= M64
    lo &= M64
    n = lo & 0xFF
    if n == LONG_MARK:
        raise ValueError("long key: bytes are not recoverable from (hi, lo)")
    return (hi.to_bytes(8, "big") + (lo >> 8).to_bytes(7, "big"))[:n]


def key_tag(hi: int, lo: int) -> int:
    return fmix64((hi & M64) ^ fmix64((lo + 0x9E3779B97F4A7C15) & M64)) | 1


def fnv1(b: bytes) -> int:
    """Exact uint32 FNV-1 (reference partitionfn, examples/WordCount/partitionfn.lua:8-16)."""
    h = FNV_OFFSET
    for c in b:
        h = ((h * FNV_PRIME) & 0xFFFFFFFF) ^ c
    return h


def fnv1_lua_double(b: bytes) -> int:
    """FNV-1 exactly as the reference computes it in Lua 5.2 doubles.

    ``h = (h * FNV_prime) % 2^32`` is evaluated in IEEE doubles, so once
    h*prime exceeds 2^53 low bits are lost; kept for parity tests.
    """
    h = float(FNV_OFFSET)
    for c in b:
        h = (h * float(FNV_PRIME)) % 4294967296.0
        h = float(int(h) ^ c)
    return int(h)


def make_rep(off: int, length: int) -> int:
    return (off << REP_LEN_BITS) | min(length, REP_LEN_MASK)


# ---------------------------------------------------------------------------
# Vectorised CPU tokenizer (reference semantics of line:gmatch("[^%s]+")).

def token_spans(buf: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Start offsets and lengths of maximal non-whitespace runs."""
    buf = np.asarray(buf, dtype=np.uint8)
    if buf.size == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    ws = _WS_TABLE[buf]
    nw = ~ws
    d = np.diff(nw.astype(np.int8), prepend=0, append=0)
    starts = np.flatnonzero(d == 1).astype(np.int64)
    ends = np.flatnonzero(d == -1).astype(np.int64)
    return starts, ends - starts


def span_keys(buf: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """(hi, lo) uint64 keys of spans; vectorised for packed keys."""
    buf = np.asarray(buf, dtype=np.uint8)
    n = starts.size
    hi = np.zeros(n, np.uint64)
    lo = np.zeros(n, np.uint64)
    if n == 0:
        return hi, lo
    padded = np.concatenate([buf, np.zeros(16, np.uint8)])
    for k in range(PACK_MAX):
        m = lens > k
        if not m.any():
            break
        b = padded[starts[m] + k].astype(np.uint64)
        if k < 8:
            hi[m] |= b << np.uint64(56 - 8 * k)
        else:
            lo[m] |= b << np.uint64(56 - 8 * (k - 8))
    short = lens <= PACK_MAX
    lo[short] |= lens[short].astype(np.uint64)
    for i in np.flatnonzero(~short):
        s, ln = int(starts[i]), int(lens[i])
        lo[i] = np.uint64(long_lo(long_hash(bytes(buf[s:s + ln]))))
    return hi, lo


def fnv1_spans(buf: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Exact uint32 FNV-1 of each span (vectorised over spans)."""
    buf = np.asarray(buf, dtype=np.uint8)
    h = np.full(starts.size, FNV_OFFSET, dtype=np.uint64)
    if starts.size == 0:
        return h.astype(np.uint32)
    maxlen = int(lens.max())
    for k in range(maxlen):
        m = lens > k
        b = buf[starts[m] + k].astype(np.uint64)
        h[m] = ((h[m] * np.uint64(FNV_PRIME)) & np.uint64(0xFFFFFFFF)) ^ b
    return h.astype(np.uint32)
