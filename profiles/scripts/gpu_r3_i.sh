#!/bin/bash
# Round-3: where the general plane's CSV group-by and bigram steps go.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_i}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_scores -o run -- python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 2 > $OUT/prof_scores.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bigram -o run -- python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 1 > $OUT/prof_bigram.log 2>&1
