#!/bin/bash
# Sparse map tables (MR_MAP_SPARSITY for ranks mapping >= MR_MAP_SPARSE_MIN_MB):
# the 1-GPU benches (staged, resident) twice, the W = 2 / 4 / 8 per-rank
# proxies, SPMD GPU tests
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sparse}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged_$i.log 2>&1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --resident --no-cold > $OUT/bench_resident_$i.log 2>&1
done
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w$w.log 2>&1
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "spmd or e2e or streaming or exactness or device" > $OUT/pytest_spmd.log 2>&1
