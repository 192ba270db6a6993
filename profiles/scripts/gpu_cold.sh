#!/bin/bash
# Exact-size pinned split buffers: cold-path probe, SPMD/e2e GPU tests, staged
# bench with the cold first iteration (x2) and the resident bench
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-cold}
mkdir -p $OUT
timeout -k 10 300 python -u tools/cold_probe.py > $OUT/cold_probe.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "spmd or e2e or streaming or exactness or device or loader or io" > $OUT/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged_$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --resident --no-cold > $OUT/bench_resident.log 2>&1
