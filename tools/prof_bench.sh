#!/bin/bash
# rocprofv3 kernel + memcpy trace of a short bench run (no PMC counters)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1
