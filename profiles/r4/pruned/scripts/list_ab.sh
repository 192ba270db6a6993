#!/bin/bash
# List-mode inserts: the LDS key -> slot cache (list_combine_kernel) vs one
# row per thread (MR_AGG_DIRECT=1), alternating, on the reducefn3 word count.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-list_ab}
mkdir -p $OUT
for i in 1 2; do
  for d in 0 1; do
    MR_AGG_DIRECT=$d timeout -k 10 200 python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 \
      --steps 10 --warmup 2 > $OUT/direct${d}_$i.log 2>&1 || exit $?
    echo "direct=$d run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/direct${d}_$i.log)"
  done
done
# list plane with pipelined iterations: its GPU tests, then the inverted-index bench
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invidx.py -m gpu \
  > $OUT/invidx_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_invidx.py --validate > $OUT/invidx_bench.log 2>&1 || exit $?
echo "invidx $(grep -o '"ms_per_step": [0-9.]*' $OUT/invidx_bench.log)"
MR_PIPELINE=0 timeout -k 10 200 python3 tools/bench_invidx.py --validate > $OUT/invidx_bench_nopipe.log 2>&1 || exit $?
echo "invidx no-pipeline $(grep -o '"ms_per_step": [0-9.]*' $OUT/invidx_bench_nopipe.log)"
# n-gram spans in one pass: their GPU tests, then the bigram bench
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_generic_gpu.py \
  -k "ngrams or tokens or generic_gpu_w1" > $OUT/ngram_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 --validate > $OUT/bigram.log 2>&1 || exit $?
echo "bigram $(grep -o '"ms_per_step": [0-9.]*\|"validated_full": [a-z]*' $OUT/bigram.log | paste -sd' ')"
