#!/bin/bash
# One rank of an 8-rank job (tools/proxy_rank.py) vs one rank alone, kernel stats of the 8-rank share
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_proxy
timeout -k 10 200 python3 tools/proxy_rank.py --of 8 > gpurun_out/proxy8.log 2>&1
timeout -k 10 200 python3 tools/proxy_rank.py --of 1 --steps 10 > gpurun_out/proxy1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_proxy -o run -- python3 tools/proxy_rank.py --of 8 --steps 6 > gpurun_out/prof_proxy.log 2>&1
