#!/bin/bash
# TeraSort bench x2 and its kernel stats
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ts}
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort_1.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort_2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ts -- python3 tools/bench_terasort.py --gb 10 --steps 2 --warmup 1 > $OUT/prof_ts.log 2>&1
