#!/bin/bash
# W=8 per-rank proxy, HBM-resident input: kernel trace + host timeline
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-w8res}
mkdir -p $OUT
MR_RESIDENT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o w8 -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/prof_w8.log 2>&1
MR_RESIDENT=1 MR_HOST_TIMELINE=1 timeout -k 10 300 python -u tools/proxy_world.py --world 8 --steps 30 > $OUT/host_timeline_w8.log 2>&1
