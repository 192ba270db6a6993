#!/bin/bash
# W=8 proxy: tile size of the small onesweep sorts (MR_SORT_SMALL_ROUNDS 4 / 8 / 16) — the tail's 8 passes over
# ~10^5 keys; sort tests at 8 and 16.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_small}
mkdir -p $OUT
for r in 8 16; do
  MR_SORT_SMALL_ROUNDS=$r timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_exactness.py tests/test_spmd_dist.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sort or exact or single_sync" > $OUT/pytest_r$r.log 2>&1 || exit $?
done
for rep in 1 2; do
  for r in 4 8 16; do
    MR_SORT_SMALL_ROUNDS=$r timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_r$r.rep$rep.log 2>&1 || exit $?
    echo "small_rounds=$r rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_r$r.rep$rep.log)"
  done
done
for r in 4 8; do
  MR_SORT_SMALL_ROUNDS=$r timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cold > $OUT/bench_r$r.log 2>&1 || exit $?
done
