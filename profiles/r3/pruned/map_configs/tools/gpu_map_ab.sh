#!/bin/bash
# resident-mode bench: device timing on/off (map config 6)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/map_ab2
mkdir -p $OUT
for i in 1 2; do for t in 1 0; do
MR_DEVICE_TIMING=$t timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/resident_timing${t}_$i.log 2>&1
done; done
