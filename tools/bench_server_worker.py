#!/usr/bin/env python
"""The reference's own deployment shape on MI355X: one server process + N
worker processes (reference README.md:43-75: 1 server + 4 workers on one
machine, 197 Europarl splits, "Server time" 49.229 s), here with the C++
coordinator in place of MongoDB and the workers' map/reduce jobs on the GPU
(device plane: HIP word-count kernels, columnar intermediate blobs).

The corpus is bench.py's synthetic Europarl shape (seed 1234) as one file per
split, so every word of the final answer is checked against the generator's
own counts (the server's finalfn dumps every (word, count) pair through
``MR_FINAL_DUMP``).  A run whose answer differs in any word is reported with
the bad words (and their FNV-1 partitions) and the tool exits non-zero.

``--dump DIR`` turns on the workers' job dumps (``MR_DEBUG_DUMP``, see
runtime/job.py): on a wrong answer every map output is checked against its
split file, every reduce input against the map output it names (crc32), and
every reduce result against its inputs — which stage lost the words.

    python tools/bench_server_worker.py [--workers 4] [--repeat 5] [--device auto|host]
                                        [--storage gridfs|shared|hbm] [--dump DIR] [--logs DIR]
"""
from __future__ import annotations

import argparse
import collections
import glob
import json
import os
import re
import shutil
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NPARTS = 15  # examples/WordCount/partitionfn.py NUM_REDUCERS
FINAL_DIR = "/tmp/lmr_sw_final"


def fnv1(b: bytes, n: int = NPARTS) -> int:
    h = 2166136261
    for c in b:
        h = (h * 16777619) & 0xFFFFFFFF
        h ^= c
    return h % n


def _load_dump(path: str) -> dict:
    import msgpack
    with open(path, "rb") as f:
        pairs = msgpack.unpackb(f.read(), raw=True, use_list=False)
    return {bytes(k): int(v) for k, v in pairs}


def diff(got: dict, want: dict, limit: int = 8) -> dict:
    missing = [k for k in want if k not in got]
    extra = [k for k in got if k not in want]
    wrong = [k for k in want if k in got and got[k] != want[k]]
    ex = lambda ks: [(k[:40].decode("utf-8", "replace"), fnv1(k), got.get(k), want.get(k)) for k in ks[:limit]]  # noqa
    return {"words_got": sum(got.values()), "words_want": sum(want.values()), "distinct_got": len(got),
            "distinct_want": len(want), "missing": len(missing), "extra": len(extra), "wrong": len(wrong),
            "ex_missing": ex(missing), "ex_extra": ex(extra), "ex_wrong": ex(wrong)}


def _cols_counts(blob: bytes) -> dict:
    from lua_mapreduce_1_amd.runtime import codec
    c = codec.decode_columnar(blob)
    off, kb, val = c["key_off"], c["key_blob"].tobytes(), c["val"]
    return {kb[int(off[i]):int(off[i + 1])]: int(val[i]) for i in range(val.size)}


def analyze(dump: str, files: list) -> dict:
    """Which stage went wrong: map outputs vs their split files, reduce inputs
    vs the map outputs they name, reduce results vs their inputs."""
    import zlib
    rx = re.compile(r"^(map|redin|redout)\.(.*)\.(\d+)\.(\d+)$")
    maps, redin, redout = {}, {}, {}
    for fn in os.listdir(dump):
        m = rx.match(fn)
        if not m:
            continue
        kind, name, pid, ns = m.group(1), m.group(2), int(m.group(3)), int(m.group(4))
        with open(os.path.join(dump, fn), "rb") as f:
            data = f.read()
        {"map": maps, "redin": redin, "redout": redout}[kind].setdefault(name, []).append((ns, pid, data))
    rep = {"map_files": len(maps), "dup_map_files": sum(len(v) > 1 for v in maps.values()), "bad_maps": [],
           "bad_partition": 0, "bad_transfers": [], "bad_reduces": []}
    pm = re.compile(r"\.P(\d+)\.M(\d+)$")
    by_job = collections.defaultdict(dict)
    for name, lst in maps.items():
        p, m = map(int, pm.search(name).groups())
        for _ns, pid, data in lst:
            cnt = _cols_counts(data)
            rep["bad_partition"] += sum(fnv1(k) != p for k in cnt)
            d = by_job[(m, pid)]
            for k, v in cnt.items():
                d[k] = d.get(k, 0) + v
    for (m, pid), got in sorted(by_job.items()):
        with open(files[m - 1], "rb") as f:
            want = dict(collections.Counter(f.read().split()))
        if got != want:
            rep["bad_maps"].append({"map": m, "pid": pid, **diff(got, want, 4)})
    latest = {name: lst[-1][2] for name, lst in maps.items()}
    for res, lst in redin.items():
        for _ns, pid, data in lst:
            agg = {}
            for line in data.decode().splitlines():
                name, size, crc = line.split("\t")
                mine = latest.get(os.path.basename(name))
                if mine is None or len(mine) != int(size) or zlib.crc32(mine) != int(crc):
                    rep["bad_transfers"].append({"reduce": res, "pid": pid, "input": name, "size": int(size),
                                                 "dumped_size": None if mine is None else len(mine)})
                if mine is not None:
                    for k, v in _cols_counts(mine).items():
                        agg[k] = agg.get(k, 0) + v
            outs = [x for x in redout.get(res, []) if x[1] == pid]
            if outs:
                got = _cols_counts(outs[-1][2])
                if got != agg:
                    rep["bad_reduces"].append({"reduce": res, "pid": pid, **diff(got, agg, 4)})
    return rep


def run_once(a, rep: int, files_dir: str, logs: str, env: dict) -> dict:
    conn = f"127.0.0.1:{a.port + rep}"
    W = "lua_mapreduce_1_amd.examples.WordCount"
    final = os.path.join(FINAL_DIR, f"final.r{rep}.msgpack")  # (large: kept out of the logs directory)
    os.makedirs(FINAL_DIR, exist_ok=True)
    if os.path.exists(final):
        os.remove(final)
    env = dict(env, MR_FINAL_DUMP=final)
    if a.dump:
        env["MR_DEBUG_DUMP"] = os.path.join(a.dump, f"r{rep}")
        shutil.rmtree(env["MR_DEBUG_DUMP"], ignore_errors=True)
    slog = open(os.path.join(logs, f"server.r{rep}.log"), "w")
    server = subprocess.Popen(
        [sys.executable, os.path.join(ROOT, "execute_server.py"), "--sleep", "2", "--poll", "0.01", "--device",
         a.device, conn, "wcbig", "lua_mapreduce_1_amd.examples.WordCountBig.taskfn", f"{W}.mapfn",
         f"{W}.partitionfn", f"{W}.reducefn", "lua_mapreduce_1_amd.examples.WordCountBig.finalfn", f"{W}.reducefn",
         a.storage, files_dir], stdout=subprocess.DEVNULL, stderr=slog, env=env)
    time.sleep(1.0)
    wlogs = [open(os.path.join(logs, f"worker{i}.r{rep}.log"), "w") for i in range(a.workers)]
    workers = [subprocess.Popen([sys.executable, os.path.join(ROOT, "execute_worker.py"), conn, "wcbig", "--poll",
                                 "0.01", "--max-iter", "1000", "--quiet"], stdout=subprocess.DEVNULL,
                                stderr=wlogs[i], env=env) for i in range(a.workers)]
    try:
        server.wait(timeout=a.timeout)
    finally:
        if server.poll() is None:
            server.kill()
        for w in workers:
            w.terminate()
        for w in workers:
            try:
                w.wait(10)
            except subprocess.TimeoutExpired:
                w.kill()
        slog.close()
        for f in wlogs:
            f.close()
    err = open(os.path.join(logs, f"server.r{rep}.log")).read()
    m = re.search(r"Server time\s+([0-9.]+)", err)
    out = {"rep": rep, "rc": server.returncode, "server_time_s": float(m.group(1)) if m else None}
    warn = []
    for i in range(a.workers):
        txt = open(os.path.join(logs, f"worker{i}.r{rep}.log")).read()
        warn += [ln for ln in txt.splitlines() if any(w in ln.lower() for w in ("warning", "error", "debug tail"))][:5]
    out["worker_warnings"] = warn
    if server.returncode != 0 or not os.path.exists(final):
        out["valid"] = False
        return out
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--storage", default="gridfs")
    ap.add_argument("--port", type=int, default=27317)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--dump", default=None, help="job dumps (MR_DEBUG_DUMP) under DIR/r<rep>, analysed on a mismatch")
    ap.add_argument("--logs", default="/tmp/lmr_sw_logs")
    ap.add_argument("--lines", type=int, default=None, help="smaller corpus (CPU tests only)")
    ap.add_argument("--words", type=int, default=None)
    a = ap.parse_args()
    import bench
    from lua_mapreduce_1_amd.utils import corpus
    lines = a.lines or corpus.EUROPARL_LINES
    words = a.words or corpus.EUROPARL_WORDS
    cdir = bench.corpus_dir(a.seed, lines, words)
    bench.ensure_corpus(cdir, a.seed, lines, words)
    files_dir = os.path.join(cdir, "files")
    files = sorted(glob.glob(os.path.join(files_dir, "*")))
    want = bench.truth_counts(cdir)
    os.makedirs(a.logs, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    runs, bad = [], 0
    for rep in range(a.repeat):
        r = run_once(a, rep, files_dir, a.logs, env)
        final = os.path.join(FINAL_DIR, f"final.r{rep}.msgpack")
        if r.get("valid") is not False:
            d = diff(_load_dump(final), want)
            os.remove(final)
            r["valid"] = d["missing"] == d["extra"] == d["wrong"] == 0
            if not r["valid"]:
                r["diff"] = d
                if a.dump:
                    r["analysis"] = analyze(os.path.join(a.dump, f"r{rep}"), files)
        if a.dump and r["valid"]:
            shutil.rmtree(os.path.join(a.dump, f"r{rep}"), ignore_errors=True)
        bad += not r["valid"]
        runs.append(r)
        print(json.dumps(r), flush=True)
    ok = [r["server_time_s"] for r in runs if r["valid"] and r["server_time_s"]]
    st = statistics.median(ok) if ok else None
    print(json.dumps({"mode": "server + workers (reference deployment)", "workers": a.workers, "device": a.device,
                      "storage": a.storage, "runs": len(runs), "valid_runs": len(runs) - bad,
                      "server_time_s_median": st, "server_times_s": [r["server_time_s"] for r in runs],
                      "words_per_s": words / st if st else None,
                      "vs_reference_server_time": 49.229152 / st if st else None}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
