#!/bin/bash
# One rank's share of a W-rank job on one GPU (tools/proxy_world.py, loopback
# collectives) at W = 2, 4, 8, and a kernel trace of the W = 8 share.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-proxy}
mkdir -p $OUT
for w in 2 4 8; do
timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w$w.log 2>&1
done
MR_PHASES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o w8 -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/prof_w8.log 2>&1
