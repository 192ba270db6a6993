"""emit.csv — the general plane's CSV row emitter — against a Python oracle:
on the CPU (the ops/text.py chain) and on the GPU (the fused kernel
mr_csv_fold, and the chain it is specified by), over rows with missing and
malformed fields, empty and long keys, CRLF endings, lines longer than a
kernel tile and a last split without a final newline."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_generic_plane import close_lists, run_engine  # noqa: E402

import csv_modules as CM  # noqa: E402

CONFIGS = [dict(key=1, values=(2, 0, None), sep=","),
           dict(key=0, values=(1, 1, None), sep=","),
           dict(key=2, values=(3, 1, None), sep="\t")]


def _splits(cfg, lines=6000, nkeys=300):
    old = (CM.KEY, CM.VALUES, CM.SEP)
    CM.KEY, CM.VALUES, CM.SEP = cfg["key"], cfg["values"], cfg["sep"]
    try:
        return CM.make_splits(seed=cfg["key"] + 7, lines=lines, nkeys=nkeys)
    finally:
        CM.KEY, CM.VALUES, CM.SEP = old


def _run(cfg, mode, device, lines):
    splits = _splits(cfg, lines)
    exp = CM.oracle(splits, cfg["key"], cfg["values"], cfg["sep"])
    eng, res, got = run_engine("csv_modules", splits, device, dict(cfg, values=list(cfg["values"]), mode=mode))
    return eng, res, got, exp


def test_csv_rows_spec():
    from lua_mapreduce_1_amd.ops import text as TX
    t = torch.frombuffer(bytearray(b"a,1.5,x\r\n,2,3\nb,zz\nc,4\nlong_key_beyond_16_bytes,-2.5"), dtype=torch.uint8)
    ks, kl, cols = TX.csv_rows(t, 0, (1, None), ",")
    keys = [bytes(t[s:s + n].tolist()) for s, n in zip(ks.tolist(), kl.tolist()) if n > 0]
    assert keys == [b"a", b"c", b"long_key_beyond_16_bytes"]
    assert cols[1] == 1
    ok = kl > 0
    assert cols[0][ok].tolist() == [1.5, 4.0, -2.5]


@pytest.mark.parametrize("cfg", CONFIGS, ids=["k1", "k0_shared", "tsv"])
def test_csv_fold_cpu(cfg):
    eng, res, got, exp = _run(cfg, "fused", torch.device("cpu"), 3000)
    assert len(exp) > 100
    assert close_lists(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fused", "chain"])
@pytest.mark.parametrize("cfg", CONFIGS, ids=["k1", "k0_shared", "tsv"])
def test_csv_fold_gpu(gpu, cfg, mode):
    eng, res, got, exp = _run(cfg, mode, gpu, 40_000)
    assert close_lists(got, exp)
    assert res.failed_maps == 0 and res.distinct_keys == len(exp)
    if mode == "fused":  # rows counted on the device: the rows the oracle kept
        assert eng.plane.map.rows == sum(v[2] for v in exp.values())


@pytest.mark.gpu
def test_csv_fold_table_overflow_gpu(gpu):
    """A table too small for the keys: the map is re-run with a larger one."""
    cfg = CONFIGS[0]
    splits = _splits(cfg, 40_000, nkeys=8000)
    exp = CM.oracle(splits, cfg["key"], cfg["values"], cfg["sep"])
    eng, res, got = run_engine("csv_modules", splits, gpu, dict(cfg, values=list(cfg["values"]), mode="fused"),
                               table_capacity=64)
    assert len(exp) > 4 * 1024
    assert close_lists(got, exp)


def _gather(eng, res):
    from lua_mapreduce_1_amd.runtime import codec
    got = {}
    for _n, cols in eng.gather_results(res):
        for k, v in codec.iter_columnar(cols):
            got[k] = list(v)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["csv", "mixed"])
def test_generic_pipelined_iterations_gpu(gpu, which):
    """Pipelined general-plane iterations (inputs prefetched, iteration q+1's
    map queued on its own stream and map state while q reduces): every
    iteration's result equals the oracle, from a first map that overflows its
    table on."""
    from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
    if which == "csv":
        cfg = CONFIGS[0]
        splits = _splits(cfg, 20_000, nkeys=3000)
        exp = CM.oracle(splits, cfg["key"], cfg["values"], cfg["sep"])
        mod, init = "csv_modules", dict(cfg, values=list(cfg["values"]), mode="fused")
    else:
        import gen_modules
        from test_generic_plane import make_data
        splits = make_data("text")
        exp = gen_modules.oracle(splits, "mixed")
        mod, init = "gen_modules", {"mode": "mixed"}
    init["nsplits"] = len(splits)
    eng = SPMDEngine(dict(taskfn=mod, mapfn=mod, partitionfn=mod, reducefn=mod, finalfn=None, init_args=init,
                          table_capacity=64), split_store=SplitStore(splits, pin=True), device=gpu)
    eng.prefetch, eng.pipeline = True, True
    steps = 4
    for k in range(steps):
        res = eng.run_iteration(prefetch_next=k < steps - 1, lookahead=steps - 1 - k)
        assert close_lists(_gather(eng, res), exp), k
        assert res.failed_maps == 0
    assert getattr(eng.plane, "_maps", [None, None])[1] is not None  # the pipelined path ran


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_text_edge_cases(dev):
    """Empty text, one token, text of only separators / newlines: tokens,
    n-grams and CSV rows agree with the definitions (no rows, no spans)."""
    from lua_mapreduce_1_amd.ops import text as TX
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    for b in (b"", b"x", b"\n\n\n", b" \t ", b",,,\n,,\n", b"a,1"):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) if b else torch.zeros(0, dtype=torch.uint8,
                                                                                           device=dev)
        st, ln = TX.tokens(t)
        toks = [b[s:s + n] for s, n in zip(st.tolist(), ln.tolist())]
        assert toks == b.split()
        st, ln = TX.ngrams(t, 2)
        grams = [b[s:s + n] for s, n in zip(st.tolist(), ln.tolist()) if n]
        assert grams == []  # no line of these holds two tokens
        ks, kl, cols = TX.csv_rows(t, 0, (1,), ",")
        keys = [b[s:s + n] for s, n in zip(ks.tolist(), kl.tolist()) if n]
        assert keys == ([b"a"] if b == b"a,1" else [])
