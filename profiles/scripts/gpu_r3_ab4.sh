#!/bin/bash
# Exact-order fix kernel + fitted tables: GPU tests of the general plane and
# exact order, the general bench, and a kernel trace of the bigram job.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_ab4}
mkdir -p $OUT/tl
timeout -k 10 400 python -u -m pytest tests/test_exact_order.py tests/test_generic_gpu.py tests/test_exactness.py tests/test_sparse_tables.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 2 > $OUT/tl.log 2>&1
