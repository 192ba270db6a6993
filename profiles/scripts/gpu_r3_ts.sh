#!/bin/bash
# TeraSort kernels: gather / tie fix-up A/B (tools/ts_ab.py), their GPU tests,
# the TeraSort bench and its kernel statistics.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_ts}
mkdir -p $OUT/prof
timeout -k 10 300 python -u -m pytest tests/test_records.py tests/test_terasort.py tests/test_exact_order.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/ts_ab.py > $OUT/ts_ab.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_terasort.py --steps 3 --warmup 1 > $OUT/prof_ts.log 2>&1
