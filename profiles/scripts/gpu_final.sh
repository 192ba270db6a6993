#!/bin/bash
# numbers for the README: 1-GPU bench (20 and 50 steps), 2/4/8-rank loopback proxies, kernel stats of the bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/final/bench_1gpu_20.log 2>&1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 > gpurun_out/final/bench_1gpu_50.log 2>&1
for w in 2 4 8; do timeout -k 10 120 python -u tools/proxy_world.py --world $w --steps 20 > gpurun_out/final/proxy_w${w}_20.log 2>&1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/final/bench_profiled.log 2>&1
