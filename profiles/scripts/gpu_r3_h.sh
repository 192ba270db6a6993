#!/bin/bash
# Round-3: fused word grouping (inverted index) + vectorized tie scan (TeraSort).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_invidx.py tests/test_streaming.py tests/test_terasort.py tests/test_records.py tests/test_generic_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ii -o run -- python3 tools/bench_invidx.py --steps 5 --warmup 2 > $OUT/prof_ii.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ts -o run -- python3 tools/bench_terasort.py > $OUT/prof_ts.log 2>&1
