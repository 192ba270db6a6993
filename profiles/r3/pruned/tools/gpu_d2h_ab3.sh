#!/bin/bash
# Driver-shaped staged bench (20 steps, 5 warm-up): MR_D2H sdma vs kernel, interleaved x3
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-d2hab3}
mkdir -p $OUT
for r in 1 2 3; do for m in sdma kernel; do
MR_D2H=$m timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/staged_${m}_$r.log 2>&1
done; done
