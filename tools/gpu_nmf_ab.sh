#!/bin/bash
# Next map queued before (1) or after (0) the tail: resident and staged bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-nmf}
mkdir -p $OUT
for r in 1; do for m in before_sync before_tail after_tail; do
MR_NEXT_MAP=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident_nmf${m}_$r.log 2>&1
done; done
for m in before_sync before_tail after_tail; do
MR_NEXT_MAP=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/staged_nmf${m}.log 2>&1
done
MR_NEXT_MAP=before_sync timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o res -- python3 bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/prof_res.log 2>&1
