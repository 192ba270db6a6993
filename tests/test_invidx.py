"""Inverted-index build (BASELINE config "inverted-index build on the same corpus
shape"): word -> sorted distinct line ids, diffed against a naive oracle on
CPU (1 rank), over gloo (2 and 3 ranks, the RCCL shuffle path with host
tensors) and on the GPU (HIP kernels; 1 rank and several ranks sharing it)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lua_mapreduce_1_amd.parallel.invidx import InvertedIndexBuilder, naive_index
from lua_mapreduce_1_amd.parallel.spmd import SplitStore
from lua_mapreduce_1_amd.utils.corpus import europarl_like, tricky_text


def _splits(seed=9):
    s = europarl_like(seed=seed, lines=3000, words=60000, vocab_size=3000, split_lines=500)
    s.append(tricky_text(np.random.default_rng(seed), 150_000))
    s.append(b"no trailing newline here")
    s.append(b"ends with space ")
    s.append(b"word word word\nword\n\n\nlast")
    return s


def test_cpu_single_rank_matches_oracle():
    splits = _splits()
    sh = InvertedIndexBuilder(SplitStore(splits, pin=False), device="cpu").build()
    exp = naive_index(splits)
    assert sh.to_host() == exp
    assert sh.num_postings == sum(len(v) for v in exp.values())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, on_gpu=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from lua_mapreduce_1_amd.parallel import dist as D
    _, _, device = D.init_from_env(backend="gloo", use_gpu=on_gpu)
    splits = _splits()
    b = InvertedIndexBuilder(SplitStore(splits, pin=on_gpu), device=device, num_reducers=7,
                             capacity=1 << 16, recv_capacity=1 << 16)
    sh = b.build()
    own_ok = all(p % world == rank for p in sh.part.cpu().tolist())
    shards = D.gather_objects(sh.to_host(), 0)
    if rank == 0:
        merged = {}
        dup = False
        for d in shards:
            for k, v in d.items():
                dup |= k in merged
                merged[k] = v
        q.put((merged == naive_index(splits), dup))
    oks = D.gather_objects(own_ok, 0)
    if rank == 0:
        q.put(all(oks))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, on_gpu=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, on_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    same, dup = q.get(timeout=300)
    owned = q.get(timeout=60)
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert same and not dup and owned


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_multi_rank_matches_oracle(world):
    _run(world)


@pytest.mark.gpu
def test_gpu_single_rank_matches_oracle(gpu):
    splits = _splits()
    b = InvertedIndexBuilder(SplitStore(splits, pin=True), device=gpu, capacity=1 << 16)
    sh = b.build()
    assert sh.docs.is_cuda
    assert sh.to_host() == naive_index(splits)
    # second build reuses the staged text and the (reset) table
    assert b.build(stage=False).to_host() == naive_index(splits)


@pytest.mark.gpu
def test_gpu_staged_pieces_and_prefetch(gpu):
    """Split-aligned pieces mapped as their copies land (line ids continue
    across pieces), and builds whose copies were prefetched into the other
    arena during the previous build's sort."""
    import torch
    splits = _splits()
    b = InvertedIndexBuilder(SplitStore(splits, pin=True), device=gpu, capacity=1 << 16)
    b.pieces = b._plan_pieces(first_mb=0.01, big_mb=0.03)
    b.events = [[torch.cuda.Event() for _ in b.pieces] for _ in range(2)]
    assert len(b.pieces) >= 3
    want = naive_index(splits)
    for i in range(4):
        assert b.build(prefetch_next=i < 3).to_host() == want
    assert b._prefetched is None


@pytest.mark.gpu
def test_gpu_long_lines_and_many_lines(gpu):
    """Lines longer than a tile / chunk, and more lines than one tile's worth."""
    rng = np.random.default_rng(4)
    words = [b"w%d" % i for i in range(500)]
    long_line = b" ".join(words[i % 500] for i in rng.integers(0, 500, 30000)) + b"\n"
    many = b"".join(b"%s %s\n" % (words[i % 500], words[(i * 7) % 500]) for i in range(40000))
    splits = [long_line, many, long_line[:70000] + b"\n" + many[:50000]]
    sh = InvertedIndexBuilder(SplitStore(splits, pin=True), device=gpu, capacity=1 << 14).build()
    assert sh.to_host() == naive_index(splits)


@pytest.mark.gpu
def test_gpu_dense_one_letter_tokens(gpu):
    """Tiles with more tokens than the map kernel buffers (one-letter words:
    up to 4096 tokens per 8 KiB tile > 2048) take the direct-write path."""
    rng = np.random.default_rng(5)
    letters = [bytes([c]) for c in b"abcdefghijklmnopqrstuvwxyz0123456789"]
    lines = [b" ".join(letters[i] for i in rng.integers(0, len(letters), int(n))) + b"\n"
             for n in rng.integers(1, 3000, 120)]
    splits = [b"".join(lines[:60]), b"".join(lines[60:])]
    sh = InvertedIndexBuilder(SplitStore(splits, pin=True), device=gpu, capacity=1 << 12).build()
    assert sh.to_host() == naive_index(splits)


@pytest.mark.gpu
def test_gpu_multi_rank_on_one_gpu(gpu):
    _run(2, on_gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 300_000, 1_500_000])
def test_gpu_sort_unique_matches_torch(gpu, n):
    """keys-only radix sort + fused two-pass unique == torch.unique (sorted)."""
    from lua_mapreduce_1_amd.ops import invidx as II
    from lua_mapreduce_1_amd.ops.primitives import sort_keys
    g = torch.Generator().manual_seed(n)
    keys = torch.randint(0, max(2, n // 3), (n,), generator=g, dtype=torch.int64) << 7
    keys |= torch.randint(0, 3, (n,), generator=g, dtype=torch.int64)
    got = II.sort_unique(keys.to(gpu), 40).cpu()
    assert torch.equal(got, torch.unique(keys))
    _, sk = sort_keys([keys.to(gpu)], bits=[40], return_keys=True, keys_only=True)
    assert torch.equal(sk.cpu(), torch.sort(keys).values)
