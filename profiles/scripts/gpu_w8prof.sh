#!/bin/bash
# cProfile of the W=8 per-rank proxy's timed iterations (host-side hot spots)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-w8prof}
mkdir -p $OUT
MR_RESIDENT=1 MR_CPROFILE=1 MR_CPROFILE_SORT=tottime timeout -k 10 300 python -u tools/proxy_world.py --world 8 --steps 200 > $OUT/cprofile_tottime.log 2>&1
MR_RESIDENT=1 MR_CPROFILE=1 MR_CPROFILE_SORT=cumtime timeout -k 10 300 python -u tools/proxy_world.py --world 8 --steps 200 > $OUT/cprofile_cumtime.log 2>&1
