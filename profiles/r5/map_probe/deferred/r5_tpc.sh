#!/bin/bash
# Word-count map: tiles per workgroup with the flush deferred by one tile
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_tpc}
mkdir -p $OUT
timeout -k 10 300 python -u tools/r5_tpc_probe.py > $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
grep tpc= $OUT/probe.log
for tpc in 1 4 2; do
  MR_WC3_TPC=$tpc timeout -k 10 200 python -u bench.py --resident --steps 20 --warmup 5 > $OUT/res_tpc$tpc.log 2>&1 || exit $?
  echo "resident tpc=$tpc $(grep -o '"ms_per_step": [0-9.]*\|"per_key_valid": [a-z]*' $OUT/res_tpc$tpc.log | tr '\n' ' ')"
done
MR_WC3_TPC=4 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_tpc4.log 2>&1 || exit $?
echo "proxy tpc=4 $(grep -o '"median": [0-9.]*' $OUT/proxy_tpc4.log)"
