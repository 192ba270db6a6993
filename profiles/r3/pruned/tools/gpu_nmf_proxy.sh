#!/bin/bash
# MR_NEXT_MAP modes on the W=8 / W=4 per-rank proxies (staged and resident)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-nmfp}
mkdir -p $OUT
for w in 8 4; do for m in before_sync after_tail; do
MR_NEXT_MAP=$m timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w${w}_$m.log 2>&1
MR_NEXT_MAP=$m MR_RESIDENT=1 timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w${w}_res_$m.log 2>&1
done; done
