#!/bin/bash
# Inverted-index job timeline: kernels and the engine's roctx ranges of a few pipelined steps (no counters).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_invidx_tl}
mkdir -p $OUT
MR_ROCTX=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv \
  -d $OUT/tl -o run -- python3 tools/bench_invidx.py --steps 6 --warmup 2 > $OUT/tl.log 2>&1
echo "rc=$?"
