#!/bin/bash
# quick A/B: 8/4/2-rank loopback proxies + 1-GPU bench
set -e
mkdir -p gpurun_out
for w in 8 4 2; do timeout -k 10 120 python -u tools/proxy_world.py --world $w --steps 20 > gpurun_out/proxy_w$w.log 2>&1; done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1
