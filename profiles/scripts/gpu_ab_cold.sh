#!/bin/bash
# Staged bench with and without the cold file-to-result first iteration, twice each (profiles/r2/cold_ab/)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abcold
mkdir -p $OUT
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/nocold_$i.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/cold_$i.log 2>&1
done
