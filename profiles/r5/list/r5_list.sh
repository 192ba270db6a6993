#!/bin/bash
# Value-list word count (reducefn3 / reducefn2): run-length postings (MR_CONST_RUNS) and the
# vector-L1 table probe (MR_AGG_L1_PROBE) — GPU tests, alternating timings, kernel stats, counters.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_list}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_generic_gpu.py tests/test_combiner_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
MR_AGG_L1_PROBE=1 MR_CONST_RUNS=0 timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py tests/test_value_rows_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_l1.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "0 0" "0 1" "1 0" "1 1"; do
    set -- $cfg
    MR_CONST_RUNS=$1 MR_AGG_L1_PROBE=$2 timeout -k 10 300 python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 10 --warmup 3 > $OUT/wc3_runs$1_l1$2.r$rep.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3,reducefn2 --steps 10 --warmup 3 --validate > $OUT/wc23_validate.log 2>&1 || exit $?
for v in 0 1; do
  MR_AGG_L1_PROBE=$v timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 --validate > $OUT/bigram_l1$v.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 2 > $OUT/ks.log 2>&1 || exit $?
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "agg_insert|agg_combine" --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 2 \
    --warmup 1 > $OUT/pmc_$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT/pmc_1 $OUT/pmc_2 $OUT/pmc_3 --kernel "agg_combine" > $OUT/summary_agg_combine.txt 2>&1
find $OUT -name "*.csv" -size +20M -delete
