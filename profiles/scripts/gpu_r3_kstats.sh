#!/bin/bash
# Kernel statistics of the round-3 final tree: rocprofv3 --kernel-trace --stats
# of the staged and resident word-count benches, TeraSort and the inverted
# index (kernel-trace only: the marker/memory-copy domains crash at exit here).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_kstats}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/staged -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/staged.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/resident -o run -- python3 -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/terasort -o run -- python3 -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/invidx -o run -- python3 -u tools/bench_invidx.py > $OUT/invidx.log 2>&1
find $OUT -name "*kernel_trace.csv" -delete
