#!/bin/bash
# roctx phase ranges (MR_ROCTX=1) + kernel trace of the 8-rank loopback proxy
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mk8
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/mk8 -o run -- python3 tools/proxy_world.py --world 8 --steps 10 > gpurun_out/mk8.log 2>&1
