#!/bin/bash
# Run-aggregated digit histograms: sort/ghist tests, plane tests, inverted-index
# and TeraSort benches, kernel stats of the inverted-index bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ghist}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_invidx.py tests/test_terasort.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ghist or sort or invidx or terasort or tail" > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --steps 5 --warmup 2 --validate > $OUT/bench_invidx.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ii -- python3 tools/bench_invidx.py --steps 5 --warmup 2 > $OUT/prof_ii.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort_2.log 2>&1
