#!/bin/bash
# Partitioned map flush: numerics tests, then the flush ablation (tools/wc_ablate6.py)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-part}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_exactness.py -m gpu -x -v --timeout 120 --timeout-method thread -k "wordcount or map_kernel" > $OUT/pytest_part.log 2>&1
timeout -k 10 300 python -u tools/wc_ablate6.py ${@:2} > $OUT/ablate6.log 2>&1
