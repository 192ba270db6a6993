"""The bigram job on the fold plane over pipelined iterations (the bench's
schedule: inputs prefetched, the next map issued during this iteration), with
the fused device tail and with the exact-order tail (which the benchmark
corpus falls back to; forced here), every iteration's counts checked against
a Python oracle."""
from __future__ import annotations

import re
from collections import Counter

import pytest

M = "lua_mapreduce_1_amd.examples.Bigram"


def _oracle(splits) -> dict:
    out: Counter = Counter()
    for s in splits:
        for line in s.split(b"\n"):
            toks = re.findall(rb"[^ \t\n\v\f\r]+", line)
            for a, b in zip(toks, toks[1:]):
                out[a + b" " + b] += 1  # (europarl_like text is single-spaced)
    return {k.decode(): v for k, v in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [True, False], ids=["exact_tail", "fused_tail"])
def test_bigram_pipelined_iterations_gpu(gpu, exact):
    from lua_mapreduce_1_amd.parallel import spmd as S
    from lua_mapreduce_1_amd.runtime import codec
    from lua_mapreduce_1_amd.utils.corpus import europarl_like
    splits = europarl_like(seed=5, lines=20_000, words=300_000, vocab_size=30_000, split_lines=2000)
    want = _oracle(splits)
    eng = S.SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M,
                            init_args={"nsplits": len(splits), "num_reducers": 7, "quiet": True}),
                       split_store=S.SplitStore(splits), device=gpu)
    eng.prefetch, eng.pipeline = True, True
    if exact:
        eng._exact_tail = True  # (set by the first fallback of the fused tail)
    steps = 5
    for k in range(steps):
        res = eng.run_iteration(prefetch_next=k < steps - 1, lookahead=steps - 1 - k)
        got = {key: v[0] for _n, c in eng.gather_results(res) for key, v in codec.iter_columnar(c)}
        assert got == want, f"iteration {k}: {len(got)} keys vs {len(want)}"
