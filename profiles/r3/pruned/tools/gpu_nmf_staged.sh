#!/bin/bash
# Host-staged headline bench, MR_NEXT_MAP before_sync vs after_tail, interleaved x3
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-nmfs}
mkdir -p $OUT
for r in 1 2 3; do for m in before_sync after_tail; do
MR_NEXT_MAP=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/staged_${m}_$r.log 2>&1
done; done
