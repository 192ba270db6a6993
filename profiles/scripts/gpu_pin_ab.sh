#!/bin/bash
# Exact-size vs torch-pool pinned split buffers, interleaved on one box: the
# staged bench (steady state + cold first iteration), three rounds
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pin_ab}
mkdir -p $OUT
for i in 1 2 3; do
  for v in 1 0; do
    MR_PIN_EXACT=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_exact${v}_$i.log 2>&1
  done
done
