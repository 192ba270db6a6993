#!/bin/bash
# Onesweep tile-size A/B: sort microbench at rounds 16/24/32 (sorts of >= 4 M
# keys), TeraSort and inverted-index benches at 16/24/32, the word-count
# benches and the sort-related GPU tests at the default
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rounds}
mkdir -p $OUT
timeout -k 10 200 python -u tools/onesweep_rounds_ab.py 16 24 32 > $OUT/rounds_ab.log 2>&1
for r in 16 24 32; do
  MR_SORT_ROUNDS=$r timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort_r$r.log 2>&1
  MR_SORT_ROUNDS=$r timeout -k 10 300 python -u tools/bench_invidx.py > $OUT/bench_invidx_r$r.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/bench_wc.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold --resident > $OUT/bench_wc_resident.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "sort or terasort or invidx or exactness or tail" > $OUT/pytest_sort.log 2>&1
