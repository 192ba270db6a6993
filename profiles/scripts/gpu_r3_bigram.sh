#!/bin/bash
# Kernel statistics of the general plane's bigram job (rocprofv3 kernel trace,
# no counters) and the bigram/scores bench itself.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_bigram}
mkdir -p $OUT/prof
timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 1 > $OUT/prof_bigram.log 2>&1
