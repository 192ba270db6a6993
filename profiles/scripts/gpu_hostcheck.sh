#!/bin/bash
# Host-overhead change check: GPU tests, W=8/W=4 proxies (staged, resident), W=8 host timeline, 1-GPU bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-hostcheck}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for w in 8 4; do
timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 40 > $OUT/proxy_w$w.log 2>&1
MR_RESIDENT=1 timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 40 > $OUT/proxy_w${w}_res.log 2>&1
done
MR_HOST_TIMELINE=1 timeout -k 10 300 python -u tools/proxy_world.py --world 8 --steps 30 > $OUT/host_timeline_w8.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_1gpu_20.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_1gpu_resident.log 2>&1
