#!/bin/bash
# Kernel trace of the inverted-index bench (timeline of a steady iteration:
# tools/copy_kernel_timeline.py --anchor ii_map).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_iitl}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/bench_invidx.py --steps 4 --warmup 2 > $OUT/run.log 2>&1
