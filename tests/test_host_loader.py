"""Native split loader (csrc/host/loader.cpp via ops/io.py) and the
per-rank SplitStore built on it: every rank reads only its own splits."""
import os

import numpy as np
import pytest
import torch

from lua_mapreduce_1_amd.ops import io as mio
from lua_mapreduce_1_amd.parallel.spmd import SplitStore, assign_contiguous


def _files(tmp_path, contents):
    paths = []
    for i, c in enumerate(contents):
        p = tmp_path / f"s{i:03d}.txt"
        p.write_bytes(c)
        paths.append(str(p))
    return paths


def test_async_load_pieces_and_padding(tmp_path):
    rng = np.random.default_rng(0)
    contents = [rng.integers(33, 127, n).astype(np.uint8).tobytes() for n in (0, 5, 3 << 20, 17, 1 << 20)]
    paths = _files(tmp_path, contents)
    lens = [len(c) for c in contents]
    off = np.concatenate([[0], np.cumsum([n + 1 for n in lens])])
    dst = torch.full((int(off[-1]),), 7, dtype=torch.uint8)
    ld = mio.AsyncLoad(paths, [0] * 5, lens, off[:-1], [1] * 5, dst, threads=4, piece=1 << 18)
    ld.wait_jobs(0, 5)
    ld.wait()
    b = dst.numpy().tobytes()
    for i, c in enumerate(contents):
        assert b[off[i]:off[i] + len(c)] == c and b[off[i] + len(c)] == 10


def test_async_load_missing_file_raises(tmp_path):
    dst = torch.zeros(16, dtype=torch.uint8)
    ld = mio.AsyncLoad([str(tmp_path / "nope")], [0], [8], [0], [0], dst)
    with pytest.raises(OSError):
        ld.wait_jobs(0, 1)


def test_async_load_short_file_raises(tmp_path):
    p = _files(tmp_path, [b"abc"])
    dst = torch.zeros(16, dtype=torch.uint8)
    with pytest.raises(OSError):
        mio.AsyncLoad(p, [0], [8], [0], [0], dst).wait()


@pytest.mark.parametrize("world", [1, 3])
def test_split_store_from_files_owns_its_share(tmp_path, world):
    rng = np.random.default_rng(1)
    contents = [b" ".join(b"w%d" % x for x in rng.integers(0, 50, int(rng.integers(1, 400)))) for _ in range(11)]
    paths = _files(tmp_path, contents)
    sizes = [len(c) + 1 for c in contents]
    for rank in range(world):
        st = SplitStore.from_files(paths, rank, world, pin=False, threads=3)
        i0, i1 = assign_contiguous(sizes, rank, world)
        assert st.own == (i0, i1) and len(st) == 11
        st.wait_ready(i0, i1)
        st.finish_loading()
        for i in range(i0, i1):
            a, b = st.region(i, i + 1)
            assert st.buffer[a:b].numpy().tobytes() == contents[i] + b"\n"
        assert st.buffer.numel() == sum(sizes[i0:i1])
        if world > 1:
            with pytest.raises(ValueError):
                st.region(0, 11)


def test_split_store_from_blob_matches_list_store(tmp_path):
    splits = [b"a b c\n", b"dd ee", b"", b"ff\n", b"g h "]
    blob = tmp_path / "blob.bin"
    blob.write_bytes(b"".join(splits))
    off = np.concatenate([[0], np.cumsum([len(s) for s in splits])])
    ref = SplitStore(splits, pin=False)
    st = SplitStore.from_blob(str(blob), off, pin=False)
    st.finish_loading()
    assert np.array_equal(st.offsets, ref.offsets)
    assert st.buffer.numpy().tobytes() == ref.buffer.numpy().tobytes()


def test_drop_page_cache(tmp_path):
    p = _files(tmp_path, [b"x" * 4096])[0]
    assert mio.drop_page_cache(p) in (True, False)
    assert mio.load_file(p).numpy().tobytes() == b"x" * 4096
