#!/bin/bash
# re-check of a freshly rebuilt tree: GPU tests, smoke(), 1-GPU bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/recheck
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/recheck/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/recheck/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/recheck/bench_1gpu_20.log 2>&1
