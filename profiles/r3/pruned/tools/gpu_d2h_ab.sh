#!/bin/bash
# Downloads by shader stores (default) vs SDMA, resident and staged bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-d2hab}
mkdir -p $OUT
for m in sdma kernel; do
MR_D2H=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident_$m.log 2>&1
done
for m in sdma kernel; do
MR_D2H=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/staged_$m.log 2>&1
done
