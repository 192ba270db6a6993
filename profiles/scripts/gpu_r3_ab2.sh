#!/bin/bash
# TeraSort A/B after the key-pass unroll; the general plane's GPU tests and
# bench after the exact-tail gathers were fused; kernel statistics of the CSV
# group-by job (general plane, typed folds).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_ab2}
mkdir -p $OUT/prof_scores
timeout -k 10 400 python -u -m pytest tests/test_records.py tests/test_terasort.py tests/test_exact_order.py tests/test_generic_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/ts_ab.py > $OUT/ts_ab.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_scores -o run -- python3 tools/bench_generic.py --jobs scores --steps 3 --warmup 1 > $OUT/prof_scores.log 2>&1
