#!/bin/bash
# Round-3: LDS-combining general fold (tests + CSV/bigram bench).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_generic_gpu.py tests/test_generic_server_worker.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 400 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
