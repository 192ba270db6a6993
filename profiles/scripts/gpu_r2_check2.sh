#!/bin/bash
# GPU tests of the new pieces + resident A/B (device timing on/off)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r2e}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_streaming.py tests/test_device_failures.py tests/test_exactness.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_new.log 2>&1
for t in 1 0; do
MR_DEVICE_TIMING=$t timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident_timing${t}.log 2>&1
done
