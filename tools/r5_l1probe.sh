#!/bin/bash
# A/B of the plain-load (vector-L1) table probe in the general plane's per-row insert
# (MR_AGG_L1_PROBE): generic GPU tests with it on, then reducefn3 / bigram alternating.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_l1probe}
mkdir -p $OUT
MR_AGG_L1_PROBE=1 timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py tests/test_value_rows_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_l1.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    MR_AGG_L1_PROBE=$v timeout -k 10 300 python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 10 --warmup 3 > $OUT/wc3_l1$v.r$rep.log 2>&1 || exit $?
  done
done
for v in 0 1; do
  MR_AGG_L1_PROBE=$v timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 --validate > $OUT/bigram_l1$v.log 2>&1 || exit $?
done
MR_AGG_L1_PROBE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_l1 -o run -- python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 2 > $OUT/prof_l1.log 2>&1 || exit $?
MR_AGG_L1_PROBE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_l0 -o run -- python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 2 > $OUT/prof_l0.log 2>&1
