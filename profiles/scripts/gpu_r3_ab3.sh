#!/bin/bash
# General plane: GPU tests, then the bigram / CSV bench with 256- and
# 512-thread combine blocks (MR_AGG_BLOCK) on the same box.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_ab3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py tests/test_generic_server_worker.py tests/test_exactness.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
MR_AGG_BLOCK=256 timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic_256.log 2>&1
MR_AGG_BLOCK=512 timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic_512.log 2>&1
MR_AGG_BLOCK=256 timeout -k 10 300 python -u tools/bench_generic.py --jobs scores > $OUT/generic_256b.log 2>&1
