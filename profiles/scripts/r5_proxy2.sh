#!/bin/bash
# W=8 proxy: staged vs HBM-resident input (is the loop copy-gated?), host timelines, kernel stats.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_proxy2}
mkdir -p $OUT
for rep in 1 2; do
  for r in 0 1; do
    MR_RESIDENT=$r timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_res$r.r$rep.log 2>&1 || exit $?
    echo "resident=$r rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_res$r.r$rep.log)"
  done
done
MR_RESIDENT=1 MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_res1_hosttl.log 2>&1 || exit $?
MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_res0_hosttl.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/ks.log 2>&1
