#!/usr/bin/env python
"""The reference's own deployment shape on MI355X: one server process + N
worker processes (reference README.md:43-75: 1 server + 4 workers on one
machine, 197 Europarl splits, "Server time" 49.229 s), here with the C++
coordinator in place of MongoDB and the workers' map/reduce jobs on the GPU
(device plane: HIP word-count kernels, columnar intermediate blobs).

Writes the Europarl-shaped splits as files (like the reference's split
directory), runs execute_server.py + N execute_worker.py, and prints the
server's statistics block and one JSON line with the server time and words/s.

    python tools/bench_server_worker.py [--workers 4] [--device auto|host]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--dir", default="/tmp/lmr_europarl_splits")
    ap.add_argument("--port", type=int, default=27317)
    a = ap.parse_args()
    from lua_mapreduce_1_amd.utils import corpus
    if not os.path.isdir(a.dir) or len(os.listdir(a.dir)) < 197:
        t = time.time()
        corpus.write_splits(corpus.europarl_like(), a.dir)
        print(f"# wrote splits in {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    conn = f"127.0.0.1:{a.port}"
    W = "lua_mapreduce_1_amd.examples.WordCount"
    out = open("/tmp/lmr_sw_final.txt", "w")
    server = subprocess.Popen(
        [sys.executable, os.path.join(ROOT, "execute_server.py"), "--sleep", "2", "--poll", "0.01", "--device",
         a.device, conn, "wcbig", "lua_mapreduce_1_amd.examples.WordCountBig.taskfn", f"{W}.mapfn",
         f"{W}.partitionfn", f"{W}.reducefn", "lua_mapreduce_1_amd.examples.WordCountBig.finalfn", f"{W}.reducefn",
         "gridfs", a.dir], stdout=out, stderr=subprocess.PIPE, text=True, env=env)
    time.sleep(1.0)
    workers = [subprocess.Popen([sys.executable, os.path.join(ROOT, "execute_worker.py"), conn, "wcbig", "--poll",
                                 "0.01", "--max-iter", "1000", "--quiet"], stdout=subprocess.DEVNULL,
                                stderr=subprocess.DEVNULL, env=env) for _ in range(a.workers)]
    try:
        _, err = server.communicate(timeout=900)
    finally:
        for w in workers:
            w.terminate()
        for w in workers:
            try:
                w.wait(10)
            except subprocess.TimeoutExpired:
                w.kill()
    out.close()
    sys.stderr.write(err[-3000:])
    m = re.search(r"Server time\s+([0-9.]+)", err)
    if server.returncode != 0 or not m:
        print(json.dumps({"ok": False, "rc": server.returncode}))
        return 1
    st = float(m.group(1))
    lines = sum(1 for _ in open("/tmp/lmr_sw_final.txt"))
    print(json.dumps({"mode": "server + workers (reference deployment)", "workers": a.workers, "device": a.device,
                      "server_time_s": st, "words_per_s": corpus.EUROPARL_WORDS / st,
                      "vs_reference_server_time": 49.229152 / st, "final_lines": lines}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
