#!/bin/bash
# host-side cost of the 8-rank loopback proxy: cProfile + roctx phase ranges with the kernel trace
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mk8
MR_CPROFILE=1 timeout -k 10 120 python3 tools/proxy_world.py --world 8 --steps 200 > gpurun_out/cprof8.log 2>&1
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/mk8 -o run -- python3 tools/proxy_world.py --world 8 --steps 20 > gpurun_out/mk8.log 2>&1
