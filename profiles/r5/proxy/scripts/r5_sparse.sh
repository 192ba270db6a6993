#!/bin/bash
# W=8 proxy: the rank's map table dense (default below 128 MiB mapped) vs sparse (MR_MAP_SPARSE_MIN_MB=0,
# MR_MAP_SPARSITY 4 / 8 / 16 slots per key): map time against the send-side compaction's slot scan.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_sparse}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "128 8" "0 4" "0 8" "0 16"; do
    set -- $cfg
    MR_MAP_SPARSE_MIN_MB=$1 MR_MAP_SPARSITY=$2 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_min$1_sp$2.r$rep.log 2>&1 || exit $?
    echo "min=$1 sp=$2 rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_min$1_sp$2.r$rep.log) $(grep -o '"device_map": [0-9.e-]*' $OUT/proxy_min$1_sp$2.r$rep.log)"
  done
done
