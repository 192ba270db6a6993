#!/bin/bash
# After the linear-time compaction scan: GPU tail/SPMD tests, benches at
# sparsity 8 / 16, proxies with sparse tables at every world size, kernel
# stats of the resident bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sparse3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "spmd or e2e or streaming or exactness or device or tail or shuffle" > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged.log 2>&1
for sp in 8 16; do
  MR_MAP_SPARSITY=$sp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --resident --no-cold > $OUT/bench_resident_s$sp.log 2>&1
done
for w in 4 8; do
  timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w$w.log 2>&1
  MR_MAP_SPARSE_MIN_MB=0 timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w${w}_sparse.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o res -- python3 bench.py --steps 20 --warmup 5 --resident --no-cold > $OUT/prof_resident.log 2>&1
