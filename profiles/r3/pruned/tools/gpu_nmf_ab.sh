#!/bin/bash
# When the next map is queued (MR_NEXT_MAP), HBM-resident bench, interleaved x2,
# plus a kernel trace of the chain mode
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-nmf}
mkdir -p $OUT
for r in 1 2; do for m in chain before_sync after_tail; do
MR_NEXT_MAP=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident_${m}_$r.log 2>&1
done; done
MR_NEXT_MAP=chain timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o res -- python3 bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/prof_res.log 2>&1
