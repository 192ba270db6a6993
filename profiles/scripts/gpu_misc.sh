#!/bin/bash
# invidx tests + bench, pipelining test over resident / next-map modes
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-misc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_invidx.py tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "invidx or pipelined or seg_gather or ghist" > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --steps 5 --warmup 2 --validate > $OUT/bench_invidx.log 2>&1
