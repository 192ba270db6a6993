#!/bin/bash
# Kernel statistics (rocprofv3 --kernel-trace --stats, no counters) of the
# final round-5 code: the headline bench, the bigram job, TeraSort.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_prof_final}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- \
  python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bigram -o run -- \
  python3 tools/bench_generic.py --jobs bigram --steps 10 --warmup 2 > $OUT/bigram.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/terasort -o run -- \
  python3 tools/bench_terasort.py > $OUT/terasort.log 2>&1 || exit $?
find $OUT -name '*kernel_stats.csv'
