"""Silent-wrong-answer guards (VERDICT r1 "what's missing" #3 / "what's weak" #3).

* Long keys (>= 16 bytes) are placed by (8-byte prefix, 56-bit hash) but their
  identity is exact: every table that matches one on (prefix, hash) compares
  the bytes.  ``ops.keys.set_long_hash_bits`` truncates the hash (a debug knob,
  host and device) so that distinct long keys collide constantly; counts must
  stay exactly those of a naive count (reference: string-equality grouping,
  job.lua:83-97, tuple.lua:250-302).
* A onesweep radix pass whose decoupled look-back gives up scatters with a
  wrong prefix; ``ops.debug_sort_fail`` forces that, and every production
  sort must detect it (re-sort or raise) instead of returning a wrong order.
"""
import os
import socket
from collections import Counter

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lua_mapreduce_1_amd import ops
from lua_mapreduce_1_amd.ops import keys as K


def colliding_text(seed: int, ntok: int = 120_000, nlong: int = 3000) -> bytes:
    """Long words that share 8-byte prefixes (so only the hash tells them
    apart), a few very long ones, and short filler words."""
    rng = np.random.default_rng(seed)
    prefixes = [b"prefixAA", b"prefixAB", b"zzzzzzzz"]
    longs = []
    seen = set()
    while len(longs) < nlong:
        p = prefixes[int(rng.integers(0, len(prefixes)))]
        n = int(rng.integers(8, 40)) if rng.random() < 0.97 else int(rng.integers(200, 3000))
        w = p + bytes(rng.integers(97, 100, n).astype(np.uint8))  # tiny alphabet: many near-duplicates
        if w not in seen:
            seen.add(w)
            longs.append(w)
    shorts = [b"a", b"bb", b"ccc", b"the", b"prefixAA", b"prefixAAbcd"]
    toks = []
    for _ in range(ntok):
        if rng.random() < 0.6:
            toks.append(longs[int(rng.zipf(1.3)) % nlong])
        else:
            toks.append(shorts[int(rng.integers(0, len(shorts)))])
    return b" ".join(toks) + b"\n"


def _table_counts(tab, src):
    hi, lo, val, rep = tab.compact()
    kb = ops.key_bytes_list(hi.cpu(), lo.cpu(), rep.cpu(), src.cpu())
    out = {}
    for k, v in zip(kb, val.cpu().tolist()):
        assert k not in out, "a key appears twice in the table"
        out[k] = v
    return out


@pytest.fixture
def collide():
    """Keep 4 (or 0) bits of the long-key hash while the test runs."""
    def set_bits(b):
        K.set_long_hash_bits(b)
    yield set_bits
    K.set_long_hash_bits(None)


@pytest.mark.parametrize("bits", [4, 0])
def test_long_key_collisions_cpu_table(collide, bits):
    collide(bits)
    text = colliding_text(1, ntok=20_000, nlong=500)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8)
    tab = ops.HashTable(1 << 14, device="cpu")
    tab.wordcount_map(t)
    assert _table_counts(tab, t) == dict(Counter(text.split()))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [4, 0])
def test_long_key_collisions_map_kernel(gpu, collide, bits):
    """The fused map (LDS combine + HBM flush + overflow path), several
    launches into one table, and a small table (long probe chains)."""
    collide(bits)
    text = colliding_text(2)
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu)
    for cap in (1 << 16, 1 << 13):
        tab = ops.HashTable(cap, device=gpu)
        cut = [0, 333_333, len(text) // 2, len(text)]
        want = Counter()
        for a, b in zip(cut[:-1], cut[1:]):
            tab.wordcount_map(t[a:b], rep_base=a, src=t)
            want.update(text[a:b].split())
        n, ovf = tab.stats()
        assert not ovf
        assert _table_counts(tab, t) == dict(want)


@pytest.mark.gpu
def test_long_key_collisions_generic_insert(gpu, collide):
    """hash_agg (emit.pairs / host pairs) and the reduce-side insert of
    received records verify bytes too."""
    collide(2)
    text = colliding_text(3, ntok=30_000, nlong=800)
    buf = np.frombuffer(text, np.uint8)
    starts, lens = K.token_spans(buf)
    hi, lo = K.span_keys(buf, starts, lens)
    rep = (starts.astype(np.uint64) << np.uint64(K.REP_LEN_BITS)) | lens.astype(np.uint64)
    dev = lambda a: torch.from_numpy(a.view(np.int64)).to(gpu)  # noqa: E731
    src = torch.from_numpy(buf.copy()).to(gpu)
    tab = ops.HashTable(1 << 15, device=gpu)
    vals = torch.ones(hi.size, dtype=torch.int64, device=gpu)
    tab.insert(dev(hi), dev(lo), vals, dev(rep), src=src)
    assert _table_counts(tab, src) == dict(Counter(text.split()))


@pytest.mark.gpu
def test_long_key_collisions_spmd_engine(gpu, collide):
    """End to end through the SPMD engine (fused tail, exact key bytes and
    byte-order fix-up of colliding long keys)."""
    collide(3)
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    splits = [colliding_text(10 + i, ntok=15_000, nlong=600) for i in range(6)]
    M = "lua_mapreduce_1_amd.models.wordcount"
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                          init_args={"nsplits": len(splits), "num_reducers": 5}),
                     split_store=SplitStore(splits), device=gpu)
    res = eng.run()
    got = {}
    for _n, cols in eng.gather_results(res):
        keys = [k for k, _ in codec.iter_columnar(cols)]
        assert keys == sorted(keys, key=lambda k: k.encode("utf-8", "surrogateescape"))
        for k, v in codec.iter_columnar(cols):
            assert k not in got
            got[k] = v[0]
    want = Counter(w.decode() for s in splits for w in s.split())
    assert got == dict(want)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shuffle_worker(port, q, backend, bits):
    """One-rank group, forced W>1 shuffle: pack -> all-to-all -> receive-side
    insert (combined layout on the GPU) with colliding long keys."""
    import datetime
    import torch.distributed as dist
    from lua_mapreduce_1_amd.ops import keys as K2
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.runtime import codec
    on_gpu = backend == "nccl"
    dist.init_process_group(backend, rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            timeout=datetime.timedelta(seconds=120),
                            **({"device_id": torch.device("cuda", 0)} if on_gpu else {}))
    K2.set_long_hash_bits(bits)
    splits = [colliding_text(20 + i, ntok=8_000, nlong=400) for i in range(4)]
    M = "lua_mapreduce_1_amd.models.wordcount"
    eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, force_shuffle=True,
                          init_args={"nsplits": len(splits), "num_reducers": 3}),
                     split_store=SplitStore(splits, pin=on_gpu),
                     device=torch.device("cuda", 0) if on_gpu else torch.device("cpu"))
    res = eng.run()
    got = {}
    for _n, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            got[k] = got.get(k, 0) + v[0]
    want = Counter(w.decode() for s in splits for w in s.split())
    q.put(got == dict(want))
    dist.destroy_process_group()


def _run_shuffle(backend, bits):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_shuffle_worker, args=(_free_port(), q, backend, bits))
    p.start()
    p.join(240)
    assert p.exitcode == 0
    assert q.get(timeout=5)


def test_long_key_collisions_shuffle_cpu():
    _run_shuffle("gloo", 2)


@pytest.mark.gpu
def test_long_key_collisions_shuffle_rccl(gpu):
    _run_shuffle("nccl", 2)


# -- radix sort look-back give-up ---------------------------------------------
@pytest.fixture
def sort_fail():
    yield ops.debug_sort_fail
    ops.debug_sort_fail(0)


@pytest.mark.gpu
def test_sort_giveup_detected_and_resorted(gpu, sort_fail):
    rng = np.random.default_rng(5)
    w = torch.from_numpy(rng.integers(-2**63, 2**63 - 1, 300_000, dtype=np.int64))
    want = ops.sort_keys([w])
    sort_fail(1)
    got = ops.sort_keys([w.to(gpu)])
    assert ops.sort_error(gpu)  # detected ...
    sort_fail(1)
    got = ops.sort_keys_checked([w.to(gpu)])  # ... and recovered by a re-sort
    assert not ops.sort_error(gpu)
    assert torch.equal(got.cpu().long(), want)
    sort_fail(100)
    with pytest.raises(RuntimeError, match="gave up"):
        ops.sort_keys_checked([w.to(gpu)], retries=2)


@pytest.mark.gpu
def test_sort_giveup_in_fused_tail(gpu, sort_fail):
    """The fused device tail packs the sort error into the 'bad' word (bit 2):
    the host re-sorts (one forced give-up: exact results) or raises (give-ups
    that do not stop)."""
    from lua_mapreduce_1_amd.parallel import spmd as S
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    splits = europarl_like(seed=4, lines=20_000, words=300_000, vocab_size=30_000, split_lines=2000)
    M = "lua_mapreduce_1_amd.models.wordcount"

    def run():
        eng = S.SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                                init_args={"nsplits": len(splits), "num_reducers": 7}),
                           split_store=S.SplitStore(splits), device=gpu)
        res = eng.run_iteration()
        return [(k, v[0]) for _n, c in eng.gather_results(res) for k, v in codec.iter_columnar(c)]

    want = dict(Counter(w.decode() for s in splits for w in s.split()))
    sort_fail(1)
    got = run()
    keys = [k for k, _ in got]
    assert len(keys) == len(set(keys)), f"{len(keys) - len(set(keys))} duplicated keys, sum {sum(v for _, v in got)}"
    assert dict(got) == want
    sort_fail(1000)
    with pytest.raises(RuntimeError, match="gave up"):
        run()


def test_engines_in_one_process_init_their_own_args():
    """Each engine is a new task: module inits run with its own init args
    (an earlier engine's nsplits must not cut a later job short)."""
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    M = "lua_mapreduce_1_amd.models.wordcount"
    for nsplits in (3, 7):
        splits = europarl_like(seed=nsplits, lines=700 * nsplits, words=5000 * nsplits, vocab_size=2000,
                               split_lines=700)
        eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                              init_args={"nsplits": len(splits), "num_reducers": nsplits}),
                         split_store=SplitStore(splits, pin=False), device="cpu")
        res = eng.run_iteration()
        assert res.total_value == 5000 * nsplits and eng.nparts == nsplits


# -- padded tail: 16-bit block histograms ----------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("bound", [255 * 16384, 64 * 65535 - 1000])
def test_padded_tail_histogram_rows_per_block(gpu, bound):
    """the padded tail's one-launch pad + histogram kernel keeps
    16-bit per-block bins.  With the grid capped at 64 blocks, a row bound
    just under 64 * 65535 gives a block 65536 rows, every sentinel row in the
    same top-digit bin: the bin wrapped and the sort's histogram was wrong.
    Both bounds (the largest the 16-bit kernel takes, and one past it that
    must use the 32-bit path) give the exact counts of a small table."""
    from lua_mapreduce_1_amd.runtime import device as dev
    rng = np.random.default_rng(3)
    words = [b"w%d" % i for i in rng.integers(0, 3000, 20_000)]
    text = b" ".join(words) + b"\n"
    ctx = dev.DeviceMapContext(gpu, "sum", 1 << 16)
    ctx.emit.words(torch.frombuffer(bytearray(text), dtype=torch.uint8).to(gpu))
    pend = dev.finalize_table_native(ctx.table, bound, ctx.source(), 7, padded=True)
    out = dev.finalize_host(pend, None, need_keys=True)
    off, blob = out["key_off"], out["key_blob"].tobytes()
    got = {blob[int(off[i]):int(off[i + 1])]: int(out["val"][i]) for i in range(out["val"].size)}
    assert got == dict(Counter(words))
    assert int(out["bounds"][-1]) == len(got)
