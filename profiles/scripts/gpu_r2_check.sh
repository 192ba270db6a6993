#!/bin/bash
# GPU tests + 1-GPU bench (with the cold file-to-result iteration) of the tree
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r2check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_1gpu_20.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_1gpu_resident.log 2>&1
