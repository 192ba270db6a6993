#!/bin/bash
# round-2 start: GPU tests + 1-GPU bench of the restored tree
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2start
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2start/pytest_gpu.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r2start/bench_1gpu_20.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --resident > gpurun_out/r2start/bench_1gpu_resident.log 2>&1
