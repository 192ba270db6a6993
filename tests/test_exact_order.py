"""ops.exact_key_perm: (partition, exact key bytes) order of mixed packed and
long keys — n-gram-like keys that share long prefixes, keys that are prefixes
of others, NUL and control bytes at the 15/16-byte boundary — against Python's
bytes order.  CPU (key words from the host helper) and GPU (mr_key_word +
onesweep rounds)."""
from __future__ import annotations

import random

import numpy as np
import pytest
import torch

from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import keys as K


def _key_set(seed: int, n: int) -> list[bytes]:
    rng = random.Random(seed)
    stems = [b"of the ", b"in the european ", b"the commission and the council ", b"x" * 15, b"abcdefghijklmnop"]
    out = set()
    while len(out) < n:
        r = rng.random()
        if r < 0.5:
            k = rng.choice(stems) + bytes(rng.choice(b"abcdefgh \t") for _ in range(rng.randrange(0, 40)))
        elif r < 0.7:
            k = rng.choice(stems)[:rng.randrange(1, 17)] + bytes(rng.choice(b"\x00\x01\x09z") for _ in
                                                                  range(rng.randrange(0, 4)))
        else:
            k = bytes(rng.randrange(1, 256) for _ in range(rng.randrange(1, 70)))
        if k:
            out.add(k)
    return sorted(out, key=lambda _: rng.random())


def _short_runs(seed: int, groups: int) -> list[bytes]:
    """Long keys in groups of 1-6 sharing their first 16 bytes (runs the
    one-kernel fix sorts), plus short keys that are prefixes of them."""
    rng = random.Random(seed)
    out = set()
    for _ in range(groups):
        pre = bytes(rng.randrange(1, 256) for _ in range(16))
        for _ in range(rng.randrange(1, 7)):
            out.add(pre + bytes(rng.randrange(0, 256) for _ in range(rng.randrange(0, 30))))
        out.add(pre[:rng.randrange(1, 16)])
    return sorted(out, key=lambda _: rng.random())


def _columns(keys: list[bytes]):
    src = np.frombuffer(b"".join(keys), np.uint8).copy()
    hi, lo, rep = [], [], []
    off = 0
    for k in keys:
        h, l_ = K.pack_key(k)
        hi.append(h)
        lo.append(l_)
        rep.append(K.make_rep(off, len(k)))
        off += len(k)
    t = lambda v: torch.from_numpy(np.array(v, dtype=np.uint64).view(np.int64))  # noqa: E731
    return t(hi), t(lo), t(rep), torch.from_numpy(src)


def _check(keys, nparts, device):
    hi, lo, rep, src = _columns(keys)
    part = torch.tensor([K.fnv1(k) % nparts for k in keys], dtype=torch.int32)
    if device is not None:
        hi, lo, rep, src, part = (x.to(device) for x in (hi, lo, rep, src, part))
    perm = ops.exact_key_perm(part, hi, lo, rep, src, nparts)
    got = [(int(part[i]), keys[i]) for i in perm.cpu().tolist()]
    assert got == sorted((int(p), k) for p, k in zip(part.cpu().tolist(), keys))


@pytest.mark.parametrize("nparts", [1, 10])
def test_exact_key_perm_cpu(nparts):
    _check(_key_set(1, 3000), nparts, None)


def test_exact_key_perm_short_only_cpu():
    _check([b"b", b"a", b"ab", b"a\x00", b"a\x00\x00", b"zz" * 7, b"zz" * 8], 1, None)


def test_exact_key_perm_short_runs_cpu():
    _check(_short_runs(3, 300), 4, None)


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [1, 10, 256])
def test_exact_key_perm_gpu(gpu, nparts):
    """Long runs of a shared 16-byte prefix: the refinement rounds."""
    _check(_key_set(2, 200_000), nparts, gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [1, 10])
def test_exact_key_perm_short_runs_gpu(gpu, nparts):
    """Runs of at most 6 keys sharing 16 bytes: one fix kernel (mr_exact_fix)."""
    _check(_short_runs(4, 40_000), nparts, gpu)


def test_exact_key_perm_returns_sorted_partitions_cpu():
    keys = _short_runs(5, 200)
    hi, lo, rep, src = _columns(keys)
    part = torch.tensor([K.fnv1(k) % 7 for k in keys], dtype=torch.int32)
    perm, spart = ops.exact_key_perm(part, hi, lo, rep, src, 7, with_part=True)
    assert torch.equal(spart, part.to(torch.int64)[perm])
    assert torch.equal(perm, ops.exact_key_perm(part, hi, lo, rep, src, 7))


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [1, 10])
def test_exact_key_perm_trailing_nul_gpu(gpu, nparts):
    """Keys past 16 bytes: the GPU sort leaves the length column out, so a
    short key and the same key followed by NUL bytes tie on the sort columns
    and the fix-up orders them (shorter first).  The partition counts come
    from the sort's histogram."""
    rng = random.Random(6)
    keys = _short_runs(6, 20_000)
    extra = []
    for k in keys[:4000]:
        stem = k[:rng.randrange(1, 14)]
        extra += [stem, stem + b"\x00", stem + b"\x00\x00", stem + b"\x00\x01"]
    keys = list(dict.fromkeys(keys + extra))
    rng.shuffle(keys)
    _check(keys, nparts, gpu)
    hi, lo, rep, src = (x.to(gpu) for x in _columns(keys))
    part = torch.tensor([K.fnv1(k) % nparts for k in keys], dtype=torch.int32, device=gpu)
    perm, spart, counts = ops.exact_key_perm(part, hi, lo, rep, src, nparts, with_part=True, with_counts=True)
    assert torch.equal(spart, part.to(torch.int64)[perm])
    assert counts.tolist() == torch.bincount(part.long().cpu(), minlength=nparts).tolist()


@pytest.mark.gpu
def test_key_meta_w1_and_gathered_lengths_gpu(gpu):
    """key_meta(want_w1=True)'s third column is key_word(..., 1); the
    lengths gather_aos4(want_len=True) derives are key_meta's."""
    keys = _key_set(7, 20_000)
    hi, lo, rep, src = (x.to(gpu) for x in _columns(keys))
    part, ln, w1 = ops.key_meta(hi, lo, rep, src, nparts=10, want_w1=True)
    p2, l2 = ops.key_meta(hi, lo, rep, src, nparts=10)
    assert torch.equal(part, p2) and torch.equal(ln, l2)
    from lua_mapreduce_1_amd.ops import primitives as P
    assert torch.equal(w1, P.key_word(hi, lo, rep, src, 1))
    aos = torch.stack([hi, lo, torch.arange(len(keys), device=gpu), rep], 1).contiguous()
    perm = torch.randperm(len(keys), device=gpu)
    g = ops.gather_aos4(perm, aos, want_len=True)
    assert torch.equal(g[0], hi[perm]) and torch.equal(g[3], rep[perm]) and torch.equal(g[4], ln[perm])


def _check_k7(keys, nparts, gpu, expect_7bit):
    hi, lo, rep, src = (x.to(gpu) for x in _columns(keys))
    part, klen, w1, k7 = ops.key_meta(hi, lo, rep, src, nparts=nparts, want_w1=True, want_k7=True)
    assert (int(k7[1][0]) == 0) == expect_7bit
    exp_part = torch.tensor([K.fnv1(k) % nparts for k in keys], dtype=torch.int32)
    assert torch.equal(part.cpu(), exp_part)
    perm, spart, counts = ops.exact_key_perm(part, hi, lo, rep, src, nparts, klen=klen, with_part=True,
                                             with_counts=True, w1=w1, k7=k7)
    got = [(int(exp_part[i]), keys[i]) for i in perm.cpu().tolist()]
    assert got == sorted((int(p), k) for p, k in zip(exp_part.tolist(), keys))
    assert torch.equal(spart.cpu(), exp_part.to(torch.int64)[perm.cpu()])
    assert counts.tolist() == torch.bincount(exp_part.long(), minlength=nparts).tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [1, 10, 256])
def test_exact_key_perm_7bit_words_gpu(gpu, nparts):
    """ASCII keys past 16 bytes (n-gram-like, shared prefixes, short keys and
    their NUL-padded twins): the 15-pass sort over the 7-bit words."""
    rng = random.Random(8)
    stems = [b"of the ", b"in the european ", b"the commission and the council ", b"x" * 15]
    keys = set()
    while len(keys) < 60_000:
        k = rng.choice(stems)[:rng.randrange(1, 40)] + bytes(rng.choice(b"abcdefgh \t~") for _ in
                                                              range(rng.randrange(0, 12)))
        keys.add(k)
        if rng.random() < 0.05:
            keys.add(k[:rng.randrange(1, 15)] + b"\x00" * rng.randrange(1, 3))
    keys = sorted(keys, key=lambda _: rng.random())
    _check_k7(keys, nparts, gpu, True)


@pytest.mark.gpu
def test_exact_key_perm_8bit_keys_fall_back_gpu(gpu):
    """A byte >= 0x80 in some key's first 16 bytes: the flag is set and the
    sort takes the byte-word columns."""
    keys = _short_runs(9, 5_000) + [b"\xff" * 20]
    _check_k7(list(dict.fromkeys(keys)), 10, gpu, False)


@pytest.mark.gpu
@pytest.mark.parametrize("alphabet", [b"ab", b"abcdefghijklmnopqrstuvwxyz ", b"0123456789abcdefghijklmnopqrstuvwxyz .",
                                      b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz .",
                                      bytes(range(32, 127))],
                         ids=["2", "27", "38", "64", "95"])
@pytest.mark.parametrize("nparts", [1, 15, 256])
def test_exact_key_perm_alphabet_words_gpu(gpu, alphabet, nparts):
    """The sort words re-coded to the byte values present (2-, 5- and 6-bit
    digits: fewer radix passes than the 7-bit words; 64 or more values: the
    7-bit words), over
    keys of 1-40 bytes with shared prefixes and NUL-padded twins."""
    rng = random.Random(len(alphabet) * 1000 + nparts)
    stems = [bytes(rng.choice(alphabet) for _ in range(rng.randrange(1, 30))) for _ in range(50)]
    keys = set()
    while len(keys) < 40_000:
        k = rng.choice(stems)[:rng.randrange(1, 30)] + bytes(rng.choice(alphabet) for _ in range(rng.randrange(0, 12)))
        keys.add(k)
        if rng.random() < 0.03:
            keys.add(k[:rng.randrange(1, 15)] + b"\x00" * rng.randrange(1, 3))
    _check_k7(sorted(keys, key=lambda _: rng.random()), nparts, gpu, True)
