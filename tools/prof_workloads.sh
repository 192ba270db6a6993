#!/bin/bash
# rocprofv3 kernel-trace stats of the secondary workloads (terasort 10 GB,
# inverted index) — no PMC counters, no runtime tracing.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_ts gpurun_out/prof_ii
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts -o run -- python3 tools/bench_terasort.py --steps 2 --warmup 1 > gpurun_out/prof_ts.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ii -o run -- python3 tools/bench_invidx.py --steps 3 --warmup 1 > gpurun_out/prof_ii.log 2>&1
