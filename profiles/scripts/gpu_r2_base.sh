#!/bin/bash
# Round-2 re-entry check: all GPU tests, the 1-GPU bench (staged and resident),
# a rocprofv3 kernel-trace of a short bench run.  Each GPU step has its own limit.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r2base}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_1gpu_20.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_1gpu_resident.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/prof_resident.log 2>&1
