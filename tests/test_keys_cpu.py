"""CPU specification of the key encoding and the CPU implementations of ops."""
import numpy as np
import torch

from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import keys as K
from lua_mapreduce_1_amd.utils.corpus import tricky_text, europarl_like


def test_pack_roundtrip_and_order():
    words = [b"a", b"ab", b"ab\0", b"ab\x01", b"abc", b"zz", b"\0", b"\xff" * 15, b"parliament", b"parliamentary",
             b"x" * 15]
    for w in words:
        hi, lo = K.pack_key(w)
        assert K.unpack_key(hi, lo) == w
    keyed = sorted(words, key=lambda w: K.pack_key(w))
    assert keyed == sorted(words)


def test_long_keys_distinct():
    a, b = b"responsibilities", b"responsibilitiez"
    ka, kb = K.pack_key(a), K.pack_key(b)
    assert ka != kb and K.is_long(ka[1]) and ka[0] == kb[0]


def test_fnv1_reference_values():
    # exact 32-bit FNV-1 of "a": (offset*prime mod 2^32) ^ 0x61
    assert K.fnv1(b"a") == ((2166136261 * 16777619) & 0xFFFFFFFF) ^ 0x61
    # the Lua-double variant agrees while h*prime < 2^53 is not guaranteed -> may differ
    assert isinstance(K.fnv1_lua_double(b"hello"), int)


def _naive(text: bytes):
    d = {}
    for w in text.split():
        d[w] = d.get(w, 0) + 1
    return d


def test_cpu_wordcount_table_matches_naive():
    rng = np.random.default_rng(0)
    text = tricky_text(rng, 100_000)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    tab = ops.HashTable(1 << 12)
    tab.wordcount_map(t)
    hi, lo, val, rep = tab.compact()
    got = dict(zip(ops.key_bytes_list(hi, lo, rep, t), val.tolist()))
    assert got == _naive(text)


def test_span_keys_vs_pack_key():
    text = b"  hello\tworld\nthisisaverylongwordindeed x\x00y \x00 " + b"q" * 15 + b" " + b"r" * 16
    buf = np.frombuffer(text, dtype=np.uint8)
    s, ln = K.token_spans(buf)
    hi, lo = K.span_keys(buf, s, ln)
    for i in range(s.size):
        w = text[s[i]:s[i] + ln[i]]
        assert (int(hi[i]), int(lo[i])) == K.pack_key(w)
    assert [text[a:a + b] for a, b in zip(s, ln)] == text.split()


def test_sort_keys_cpu_unsigned():
    w = torch.tensor([-1, 0, 5, -(2**63)], dtype=torch.int64)
    p = ops.sort_keys([w])
    assert w[p].tolist() == [0, 5, -(2**63), -1]


def test_europarl_like_shape_small():
    splits = europarl_like(seed=1, lines=25_000, words=600_000, vocab_size=20_000)
    assert len(splits) == 3
    assert sum(s.count(b"\n") for s in splits) == 25_000
    assert sum(len(s.split()) for s in splits) == 600_000
