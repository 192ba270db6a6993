#!/bin/bash
# Bigram job timeline: kernels and the
# engine's roctx ranges of a few pipelined steps (no counters; --memory-copy-trace
# crashes on the SDMA downloads' shared completion signal: "bad original signal value").
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_bigram_tl}
mkdir -p $OUT
MR_ROCTX=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv \
  -d $OUT/tl -o run -- python3 tools/bench_generic.py --jobs bigram --steps 4 --warmup 2 > $OUT/tl.log 2>&1
echo "rc=$?"
find $OUT/tl -name '*.csv' | head -20
