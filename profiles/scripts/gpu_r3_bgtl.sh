#!/bin/bash
# Kernel trace of the bigram job (timeline of one
# steady iteration: tools/host_gpu_timeline.py).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_bgtl}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 2 > $OUT/run.log 2>&1
