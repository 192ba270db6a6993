#!/bin/bash
# After a tail-kernel change: all GPU tests, the W=8 per-rank proxy, the 1-GPU bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tailcheck}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for w in 8 4; do
timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w$w.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_1gpu_20.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_1gpu_resident.log 2>&1
timeout -k 10 200 python -u tools/map_warm_probe.py 8 > $OUT/map_warm_w8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o w8 -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/prof_w8.log 2>&1
