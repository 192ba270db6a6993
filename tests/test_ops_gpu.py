"""HIP kernels vs the NumPy (CPU) implementation of the same op."""
import numpy as np
import pytest
import torch

from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import keys as K
from lua_mapreduce_1_amd.utils.corpus import tricky_text, europarl_like

pytestmark = pytest.mark.gpu


def _wc_dict(hi, lo, val, rep, src):
    kb = ops.key_bytes_list(hi.cpu(), lo.cpu(), rep.cpu(), src.cpu())
    return dict(zip(kb, val.cpu().tolist()))


def _naive(text: bytes):
    d = {}
    for w in text.split():
        d[w] = d.get(w, 0) + 1
    return d


@pytest.mark.parametrize("seed,nbytes", [(0, 1000), (1, 70_000), (2, 300_001), (3, 2_000_000)])
def test_wordcount_map_matches_naive(gpu, seed, nbytes):
    rng = np.random.default_rng(seed)
    text = tricky_text(rng, nbytes)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 16, device=gpu)
    tab.wordcount_map(t)
    hi, lo, val, rep = tab.compact()
    got = _wc_dict(hi, lo, val, rep, t)
    assert got == _naive(text)


def test_wordcount_map_unaligned_and_chunks(gpu):
    rng = np.random.default_rng(7)
    text = tricky_text(rng, 500_000)
    base = torch.frombuffer(bytearray(b"x" + text), dtype=torch.uint8).to(gpu)
    t = base[1:]  # misaligned view
    for tt in (t, t.contiguous()):
        tab = ops.HashTable(1 << 15, device=gpu)
        tab.wordcount_map(tt)
        hi, lo, val, rep = tab.compact()
        assert _wc_dict(hi, lo, val, rep, tt) == _naive(text)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wordcount_map3_launches_match_naive(gpu, seed):
    """The map kernel on tricky bytes (long tokens crossing tiles, all
    whitespace kinds, NULs), aligned and misaligned, in several launches into
    one table (per-launch overflow counters)."""
    rng = np.random.default_rng(100 + seed)
    text = tricky_text(rng, 700_001)
    base = torch.frombuffer(bytearray(b"x" + text), dtype=torch.uint8).to(gpu)
    for t in (base[1:].contiguous(), base[1:]):
        tab = ops.HashTable(1 << 16, device=gpu)
        cut = [0, 12_345, 400_000, len(text)]
        for a, b in zip(cut[:-1], cut[1:]):  # a token cut by a launch boundary counts as two
            tab.wordcount_map(t[a:b], rep_base=a)
        hi, lo, val, rep = tab.compact()
        got = _wc_dict(hi, lo, val, rep, t)
        want = {}
        for a, b in zip(cut[:-1], cut[1:]):
            for w, c in _naive(text[a:b]).items():
                want[w] = want.get(w, 0) + c
        assert got == want


def test_wordcount_europarl_like_shape(gpu):
    splits = europarl_like(seed=5, lines=20_000, words=500_000, vocab_size=50_000)
    text = b"".join(splits)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 17, device=gpu)
    tab.wordcount_map(t)
    n, ovf = tab.stats()
    assert not ovf
    hi, lo, val, rep = tab.compact()
    assert int(val.sum()) == 500_000
    assert _wc_dict(hi, lo, val, rep, t) == _naive(text)


def test_tokenize_matches_cpu(gpu):
    rng = np.random.default_rng(11)
    text = tricky_text(rng, 200_000)
    tc = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    g = ops.tokenize(tc.to(gpu))
    c = ops.tokenize(tc)
    og = np.argsort(g[2].cpu().numpy())
    for a, b in zip(g, c):
        assert np.array_equal(a.cpu().numpy()[og], b.numpy())


def test_sort_keys_matches_lexsort(gpu):
    rng = np.random.default_rng(3)
    n = 300_001
    w0 = torch.from_numpy(rng.integers(0, 7, n).astype(np.int64))
    w1 = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))
    w1[1::5] = w1[::5][: w1[1::5].numel()]  # duplicates exercise stability
    w2 = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))
    pg = ops.sort_keys([w0.to(gpu), w1.to(gpu), w2.to(gpu)], bits=[8, 64, 64]).cpu().long()
    pc = ops.sort_keys([w0, w1, w2], bits=[8, 64, 64])
    assert torch.equal(pg, pc)


def test_scan_and_bincount(gpu):
    rng = np.random.default_rng(4)
    for n in (1, 4095, 4096, 16_385, 70_001, 131_072, 131_073, 3_000_000):  # small, mid (one launch), large
        x = torch.from_numpy(rng.integers(0, 50, n).astype(np.int64))
        o, tot = ops.exclusive_scan(x.to(gpu))
        oc, tc = ops.exclusive_scan(x)
        assert torch.equal(o.cpu(), oc) and int(tot) == int(tc)
        x32 = x.to(torch.int32)
        o, tot = ops.exclusive_scan(x32.to(gpu))
        assert torch.equal(o.cpu().long(), oc) and int(tot) == int(tc)
    ids = torch.from_numpy(rng.integers(0, 37, 100_000).astype(np.int32))
    assert torch.equal(ops.bincount(ids.to(gpu), 37).cpu(), ops.bincount(ids, 37))


def test_reduce_by_key(gpu):
    rng = np.random.default_rng(9)
    n = 200_000
    hi = torch.from_numpy(np.sort(rng.integers(0, 5000, n)).astype(np.int64))
    lo = torch.from_numpy((hi.numpy() % 3).astype(np.int64))
    v = torch.from_numpy(rng.integers(-100, 100, n).astype(np.int64))
    for op in ("sum", "min", "max"):
        g = ops.reduce_by_key(hi.to(gpu), lo.to(gpu), v.to(gpu), op)
        c = ops.reduce_by_key(hi, lo, v, op)
        for a, b in zip(g, c):
            if b is not None:
                assert torch.equal(a.cpu(), b)


def test_key_meta_and_gather(gpu):
    rng = np.random.default_rng(12)
    text = tricky_text(rng, 100_000)
    tc = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    tab = ops.HashTable(1 << 14)
    tab.wordcount_map(tc)
    hi, lo, val, rep = tab.compact()
    pg, lg = ops.key_meta(hi.to(gpu), lo.to(gpu), rep.to(gpu), tc.to(gpu), nparts=15)
    pc, lc = ops.key_meta(hi, lo, rep, tc, nparts=15)
    assert torch.equal(pg.cpu(), pc) and torch.equal(lg.cpu(), lc)
    og, bg = ops.gather_key_bytes(hi.to(gpu), lo.to(gpu), rep.to(gpu), tc.to(gpu))
    oc, bc = ops.gather_key_bytes(hi, lo, rep, tc)
    assert torch.equal(og.cpu(), oc) and torch.equal(bg.cpu(), bc)


def test_hash_agg_pairs(gpu):
    rng = np.random.default_rng(13)
    n = 500_000
    hi = torch.from_numpy(rng.integers(0, 1000, n).astype(np.int64))
    lo = torch.from_numpy((rng.integers(0, 4, n) * 256 + 3).astype(np.int64))
    v = torch.from_numpy(rng.integers(1, 10, n).astype(np.int64))
    for op in ("sum", "min", "max"):
        tg = ops.HashTable(1 << 14, device=gpu, op=op)
        tg.insert(hi.to(gpu), lo.to(gpu), v.to(gpu))
        a = tg.compact()
        tc = ops.HashTable(1 << 14, op=op)
        tc.insert(hi, lo, v)
        b = tc.compact()
        pa = ops.sort_keys([a[0].cpu(), a[1].cpu()])
        ga = {(int(x), int(y)): int(z) for x, y, z in zip(a[0].cpu()[pa], a[1].cpu()[pa], a[2].cpu()[pa])}
        gb = {(int(x), int(y)): int(z) for x, y, z in zip(b[0], b[1], b[2])}
        assert ga == gb


@pytest.mark.parametrize("n", [1, 4095, 4097, 100_000, 2_000_003, 4_500_007])
def test_sort_onesweep(gpu, n):
    rng = np.random.default_rng(n)
    w0 = torch.from_numpy(rng.integers(0, 10, n).astype(np.int64))
    w1 = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))
    w1[1::3] = 42  # many ties + a uniform-ish digit pattern
    pg = ops.sort_keys([w0.to(gpu), w1.to(gpu)], bits=[8, 64]).cpu().long()
    pc = ops.sort_keys([w0, w1], bits=[8, 64])
    assert torch.equal(pg, pc)
    from lua_mapreduce_1_amd.ops.primitives import sort_error
    assert not sort_error(gpu)


@pytest.mark.parametrize("runlen", [3, 200])
def test_sort_by_partition_key(gpu, runlen):
    rng = np.random.default_rng(runlen)
    n = 50_000
    hi = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    hi[: runlen * 20] = (hi[: runlen * 20] & ~0xFF) | 0  # ...
    hi[: runlen * 20] = np.repeat(rng.integers(-2**63, 2**63 - 1, 20, dtype=np.int64), runlen)
    hi[: runlen * 20] ^= rng.integers(0, 256, runlen * 20)  # same top 7 bytes, different low byte
    lo = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    part = rng.integers(0, 3, n).astype(np.int32)
    part[: runlen * 20] = 1
    val = np.arange(n, dtype=np.int64)
    t = [torch.from_numpy(x) for x in (part, hi, lo, val, val.copy())]
    g = ops.sort_by_partition_key(*[x.to(gpu) for x in t], 3)
    c = ops.sort_by_partition_key(*t, 3)
    bad = int(g[5].item())
    if runlen > 64:
        assert bad == 1
    else:
        assert bad == 0
        for a, b in zip(g[:5], c[:5]):
            assert torch.equal(a.cpu().long(), b.long())


def test_finalize_long_tie_runs(gpu):
    from lua_mapreduce_1_amd.runtime import device as dv
    words = [b"abcdefg" + bytes([65 + i % 26, 97 + i // 26]) for i in range(300)] + [b"x", b"y", b"abcdefgh" * 3]
    text = b" ".join(words * 2) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 12, device=gpu)
    tab.wordcount_map(t)
    hi, lo, val, rep = tab.compact()
    cols = dv.finalize(hi, lo, val, rep, t, 1)
    blob = cols["key_blob"].tobytes()
    keys = [blob[cols["key_off"][i]:cols["key_off"][i + 1]] for i in range(len(cols["val"]))]
    assert keys == sorted(set(words))
    assert set(cols["val"].tolist()) == {2}


def test_device_long_key_order_without_host_fix(gpu):
    """Long keys sharing 8-byte prefixes (and packed keys with the same
    prefix) come out in exact bytewise order from the device tie fix-up; the
    host fallback flag (bit 1) is not raised."""
    rng = np.random.default_rng(5)
    pre = [b"internat", b"responsi", b"abcdefgh"]
    words = set()
    for p in pre:
        for _ in range(20):
            tail = bytes(rng.integers(97, 123, int(rng.integers(0, 14))).astype(np.uint8))
            words.add(p + tail)
    words |= {b"a", b"zz", b"internat", b"internatio"}
    words = sorted(words)
    text = b" ".join(words * 3) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 12, device=gpu)
    tab.wordcount_map(t)
    hi, lo, val, rep = tab.compact()
    part = torch.zeros(hi.numel(), dtype=torch.int32, device=gpu)
    p2, h2, l2, v2, r2, bad = ops.sort_by_partition_key(part, hi, lo, val, rep, 1, src=t)
    assert int(bad.item()) & 2 == 0
    off, blob = ops.gather_key_bytes(h2, l2, r2, t)
    off, blob = off.cpu().numpy(), blob.cpu().numpy().tobytes()
    got = [blob[off[i]:off[i + 1]] for i in range(h2.numel())]
    assert got == words


@pytest.mark.parametrize("rounds", [16, 24, 32])
def test_sort_onesweep_large_tile_sizes(gpu, rounds):
    """Sorts of >= 4 M keys with every instantiated tile size (MR_SORT_ROUNDS
    keys per thread): permutation and sorted top bits equal the CPU sort's."""
    from lua_mapreduce_1_amd.ops import _hip
    from lua_mapreduce_1_amd.utils.config import TUNABLES
    rng = np.random.default_rng(rounds)
    n = (1 << 22) + 12_345
    w = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))
    w[::7] = w[3]  # ties keep their input order (stability)
    assert _hip.lib().mr_sort_set_rounds(rounds) == 0
    try:
        pg, kg = ops.sort_keys([w.to(gpu)], bits=[64], return_keys=True, from_bit=32)
        assert not ops.sort_error(gpu)
    finally:
        _hip.lib().mr_sort_set_rounds(TUNABLES.sort_rounds)
    pc = ops.sort_keys([w >> 32 & 0xFFFFFFFF], bits=[32])
    assert torch.equal(pg.cpu().long(), pc)
    assert torch.equal(kg.cpu(), w[pc])


@pytest.mark.parametrize("resident", [False, True])
def test_spmd_prefetch_pipelined_iterations_match(gpu, monkeypatch, resident):
    """Iterations whose input copies were prefetched into the other arena give
    the same results as non-pipelined ones (and the counts stay exact); also
    with HBM-resident input (the next map queued before this map's sync,
    gated on its completion).  The first map grows the later maps' tables to
    the sparse capacity (MR_MAP_SPARSE_MIN_MB=0, 64 slots per key: past the
    default 2^20), also while a map is queued ahead."""
    import dataclasses
    from lua_mapreduce_1_amd.parallel import spmd as S
    monkeypatch.setattr(S, "TUNABLES", dataclasses.replace(S.TUNABLES, map_sparse_min_mb=0.0, map_sparsity=64))
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    M = "lua_mapreduce_1_amd.models.wordcount"
    splits = europarl_like(seed=3, lines=20_000, words=400_000, vocab_size=20_000, split_lines=1000)
    params = dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                  init_args={"nsplits": len(splits), "num_reducers": 10})
    eng = SPMDEngine(params, device=gpu, split_store=SplitStore(splits))
    eng.resident = resident
    ref = eng.run_iteration()
    ref_total, ref_keys = ref.total_value, ref.distinct_keys
    from lua_mapreduce_1_amd.runtime import codec
    want = {k: v[0] for _n, cols in eng.gather_results(ref) for k, v in codec.iter_columnar(cols)}
    assert sum(want.values()) == 400_000
    eng.prefetch = True
    for i in range(5):
        r = eng.run_iteration(prefetch_next=i < 4, lookahead=4 - i)
        assert r.total_value == ref_total == 400_000 and r.distinct_keys == ref_keys
    assert not eng._inflight
    # pipelined: the next iteration's map is queued on the other stream/table
    # while this one finalizes; every result is identical to the reference
    eng.pipeline = True
    for i in range(6):
        r = eng.run_iteration(prefetch_next=i < 5, lookahead=5 - i)
        assert r.total_value == ref_total and r.distinct_keys == ref_keys
        got = {k: v[0] for _n, cols in eng.gather_results(r) for k, v in codec.iter_columnar(cols)}
        assert got == want
    assert eng._pending is None and not eng._inflight
    want_cap = ops.next_pow2(64 * ref_keys)
    assert want_cap > 1 << 20 and all(t is not None and t.cap == want_cap for t in eng.tables)  # both slots grew


@pytest.mark.parametrize("W", [1, 3, 8])
def test_pack_by_dest_matches_cpu(gpu, W):
    """Per destination, the GPU pack holds the same (key bytes, value) set as
    the CPU specification, and absolute reps index the right bytes."""
    from lua_mapreduce_1_amd.ops import shuffle as SH
    rng = np.random.default_rng(W)
    words = [bytes(rng.integers(97, 123, int(rng.integers(1, 30))).astype(np.uint8)) for _ in range(3000)]
    text = b" ".join(words) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    tab = ops.HashTable(1 << 13, device=gpu)
    tab.wordcount_map(t.to(gpu))
    hi, lo, val, rep = tab.compact()
    part, _ = ops.key_meta(hi, lo, rep, t.to(gpu), nparts=10)
    rg, bg, xg = SH.pack_by_dest(hi, lo, val, rep, part, W, t.to(gpu), extra=7)
    rc, bc, xc = SH.pack_by_dest(hi.cpu(), lo.cpu(), val.cpu(), rep.cpu(), part.cpu(), W, t, extra=7)
    assert torch.equal(xg.cpu(), xc)
    x = xc.view(W, 3).numpy()
    rows = x[:, 0].tolist()
    nb = x[:, 1].tolist()

    def per_dest(rec, blob):
        # rebuild (bytes, val) per destination as a receiver would (one source)
        reps = SH.absolute_reps(rec, rows, nb).cpu().numpy()
        b = blob.cpu().numpy().tobytes()
        out, r0 = [], 0
        for d in range(W):
            s = set()
            for i in range(r0, r0 + rows[d]):
                off, ln = int(reps[i]) >> 24, int(reps[i]) & 0xFFFFFF
                s.add((b[off:off + ln], int(rec[i, 2])))
            out.append(s)
            r0 += rows[d]
        return out
    assert per_dest(rg.cpu(), bg[:sum(nb)]) == per_dest(rc, bc)


@pytest.mark.parametrize("W", [1, 3, 8])
def test_combined_pack_and_receive_insert(gpu, W):
    """Combined one-buffer shuffle layout: destination d's segment, received W
    times (as from W identical peers), folds into a table holding exactly the
    keys of partitions p % W == d with W times their counts and rep words that
    index the received buffer."""
    from lua_mapreduce_1_amd.ops import shuffle as SH
    rng = np.random.default_rng(40 + W)
    words = [bytes(rng.integers(97, 123, int(rng.integers(1, 30))).astype(np.uint8)) for _ in range(5000)]
    text = b" ".join(words) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 14, device=gpu)
    tab.wordcount_map(t)
    hi, lo, val, rep = tab.compact()
    part, _ = ops.key_meta(hi, lo, rep, t, nparts=10)
    src_dict = _wc_dict(hi, lo, val, rep, t)
    pmap = dict(zip(ops.key_bytes_list(hi.cpu(), lo.cpu(), rep.cpu(), t.cpu()), part.cpu().tolist()))
    buf, xchg = SH.pack_by_dest_combined(hi, lo, val, rep, part, W, t, extra=5)
    x = xchg.view(W, 3).cpu().tolist()
    assert all(r[2] == 5 for r in x) and sum(r[0] for r in x) == hi.numel()
    seg = [SH.seg_bytes(r[0], r[1]) for r in x]
    starts = np.concatenate([[0], np.cumsum(seg)]).astype(np.int64)
    for d in range(W):
        segd = buf[int(starts[d]):int(starts[d + 1])]
        rbuf = segd.repeat(W).contiguous()
        recv = torch.tensor([x[d]] * W, dtype=torch.int64, device=gpu).contiguous()
        red = ops.HashTable(1 << 14, device=gpu)
        red.insert_received(rbuf, recv, W, rows=W * x[d][0])
        rh, rl, rv, rr = red.compact()
        got = _wc_dict(rh, rl, rv, rr, rbuf)
        want = {k: W * v for k, v in src_dict.items() if pmap[k] % W == d}
        assert got == want


@pytest.mark.parametrize("nparts", [1, 10, 256])
def test_fused_tail_matches_unfused(gpu, nparts):
    from lua_mapreduce_1_amd.runtime import device as dv
    from lua_mapreduce_1_amd.utils.corpus import tricky_text
    rng = np.random.default_rng(nparts)
    text = tricky_text(rng, 400_000) + b" " + b" ".join(
        bytes(rng.integers(97, 123, int(rng.integers(1, 24))).astype(np.uint8)) for _ in range(20000)) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 16, device=gpu)
    tab.wordcount_map(t)
    n, _ = tab.stats()
    # the one-call native tail (mr_tail_run) against the unfused path
    # (compact, partition, sort, key bytes as separate ops), twice (the
    # second run reuses its cached workspace and the blob-size estimate)
    hi, lo, val, rep = tab.compact()
    b = dv.finalize(hi, lo, val, rep, t, nparts)
    b = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in b.items()}  # (pinned-pool aliases)
    for _ in range(2):
        a = dv.finalize_host(dv.finalize_table_native(tab, n, t, nparts))
        assert np.array_equal(a["bounds"], b["bounds"])
        assert np.array_equal(a["val"], b["val"])
        assert np.array_equal(np.asarray(a["key_off"], np.int64), np.asarray(b["key_off"], np.int64))
        assert a["key_blob"].tobytes() == b["key_blob"].tobytes()


@pytest.mark.parametrize("nbytes", [1, 37, 4096, 5 << 20])
def test_downloads_and_host_waits(gpu, nbytes):
    """mr_d2h_async (SDMA copy into pinned memory) + wait_stream (spin on
    the completion word) deliver exactly the device bytes, also behind a
    queued kernel and with large H2D copies in flight on another stream."""
    from lua_mapreduce_1_amd.ops import _hip
    from lua_mapreduce_1_amd.runtime import device as devmod
    g = torch.Generator(device="cpu").manual_seed(nbytes)
    src_h = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g)
    d = src_h.to(gpu)
    big_h = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    big_d = torch.empty_like(big_h, device=gpu)
    cs = torch.cuda.Stream(gpu)
    _hip.call("mr_memcpy_async", _hip.ptr(big_d), _hip.ptr(big_h), big_h.numel(), 1, _hip.stream_ptr(cs))
    d.add_(1)  # a kernel the download must wait for
    out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    devmod.dma_to_host(out, d)
    _hip.wait_stream(gpu)
    assert torch.equal(out, src_h + 1)
    # small reads of typed tensors
    t = torch.arange(3 * 8, dtype=torch.int64, device=gpu).view(2, 4, 3) * 7
    assert np.array_equal(ops.host_read(t), t.cpu().numpy())
    torch.cuda.synchronize()


def test_h2d_pull_matches_copy(gpu):
    from lua_mapreduce_1_amd.ops import _hip
    n = (3 << 20) + 45
    h = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory()
    d = torch.zeros(n, dtype=torch.uint8, device=gpu)
    _hip.call("mr_h2d_pull", _hip.ptr(d), _hip.ptr(h), n, 512, _hip.stream(gpu))
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), h)


@pytest.mark.parametrize("n,runs", [(1, True), (63, True), (64 * 1000 + 37, True), (3_000_001, True),
                                    (3_000_001, False)])
def test_radix_ghist8_matches_numpy(gpu, n, runs):
    """Digit histograms (csrc/hip/sort.hip rs_ghist8_kernel, run-aggregated
    per wave) against numpy: keys with long runs of equal digits (posting
    keys in text order; runs crossing wave boundaries, a partial last wave)
    and random keys."""
    from lua_mapreduce_1_amd.ops import _hip
    rng = np.random.default_rng(n)
    if runs:
        lens = rng.integers(1, 90, n // 3 + 2)
        vals = rng.integers(0, 2**62, lens.size, dtype=np.int64)
        k = np.repeat(vals, lens)[:n]
        k[::7] ^= rng.integers(0, 256, k[::7].size)  # break some runs in the low digit only
    else:
        k = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    keys = torch.from_numpy(k).to(gpu)
    # 0x100: run-aggregated (MR_GHIST_RUNS); bits 16-23: first digit
    for flags in (8 | 0x100, 3 | 0x100, 8, 3, 8 | (4 << 16), 8 | 0x100 | (5 << 16)):
        gh = torch.zeros(2048, dtype=torch.int32, device=gpu)
        _hip.call("mr_radix_ghist8", _hip.ptr(keys), n, _hip.ptr(gh), flags, _hip.stream(gpu))
        ndig, d0 = flags & 0xFF, (flags >> 16) & 0xFF
        got = gh.cpu().numpy().reshape(8, 256)
        ku = k.view(np.uint64)
        for b in range(8):
            want = np.bincount(((ku >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.int64), minlength=256) \
                if d0 <= b < ndig else np.zeros(256, np.int64)
            assert np.array_equal(got[b], want), b


@pytest.mark.parametrize("nparts", [1, 7])
def test_tail_orders_long_runs_of_a_shared_prefix_exactly(gpu, nparts):
    """Keys that share their first 8 bytes in runs far longer than the tie
    fix-up handles (n-gram-like: one long prefix, many suffixes, long keys
    among them): the tail falls back to the exact device order (key words +
    length), no host sort — result keys are in bytewise order in every
    partition with their counts."""
    from lua_mapreduce_1_amd.runtime import device as dv
    rng = np.random.default_rng(nparts)
    words = set()
    while len(words) < 6000:
        k = int(rng.integers(0, 24))
        words.add(b"sharedpx" + bytes(rng.integers(97, 100, k).astype(np.uint8)))
    words = sorted(words)
    reps = rng.integers(1, 4, len(words))
    toks = [w for w, r in zip(words, reps) for _ in range(int(r))]
    rng.shuffle(toks)
    text = b" ".join(toks) + b"\n"
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    tab = ops.HashTable(1 << 15, device=gpu)
    tab.wordcount_map(t)
    n, _ = tab.stats()
    c = dv.finalize_host(dv.finalize_table_native(tab, n, t, nparts))
    kb = c["key_blob"].tobytes()
    ko = np.asarray(c["key_off"], np.int64)
    want = dict(zip(words, reps.tolist()))
    got = {}
    for p in range(nparts):
        a, b = int(c["bounds"][p]), int(c["bounds"][p + 1])
        keys = [kb[ko[i]:ko[i + 1]] for i in range(a, b)]
        assert keys == sorted(keys)
        got.update(zip(keys, c["val"][a:b].tolist()))
    assert got == want
