#!/bin/bash
# Round-1 checkpoint: GPU tests, W = 8/4/2 proxies (shader and SDMA downloads), 1-GPU bench
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for w in 8 4 2; do timeout -k 10 120 python -u tools/proxy_world.py --world $w --steps 20 > gpurun_out/proxy_w$w.log 2>&1; done
MR_D2H=sdma timeout -k 10 120 python -u tools/proxy_world.py --world 8 --steps 20 > gpurun_out/proxy_w8_sdma.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1
