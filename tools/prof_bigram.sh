#!/bin/bash
# Bigram job timeline: kernels (per queue) and the engine's roctx phase ranges
# of a few pipelined steps (no counters in this run).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bigram_tl}
mkdir -p $OUT
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/tl -o run -- \
  python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 2 > $OUT/tl.log 2>&1
