#!/bin/bash
# Round 5: TeraSort with 8-bit (4 passes) vs 11-bit (3 passes) u32 prefix sorts, and the sort11 unit test
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_terasort}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_records.py -m gpu -x -v -k sort11 --timeout 200 --timeout-method thread > $OUT/pytest_sort11.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_terasort.py > $OUT/ts_d8.log 2>&1 || exit $?
for r in 8 16 32; do
  MR_SORT32_DIGIT_BITS=11 MR_SORT11_ROUNDS=$r timeout -k 10 200 python -u tools/bench_terasort.py > $OUT/ts_d11_r$r.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_d8 -o run -- python3 tools/bench_terasort.py --steps 3 --warmup 1 > $OUT/prof_d8.log 2>&1 || exit $?
MR_SORT32_DIGIT_BITS=11 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_d11 -o run -- python3 tools/bench_terasort.py --steps 3 --warmup 1 > $OUT/prof_d11.log 2>&1 || exit $?
# counters of the 11-bit passes (kernel-trace free, one group per run): LDS bank conflicts and wave waits
MR_SORT32_DIGIT_BITS=11 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "onesweep|hist11" --output-format csv -d $OUT/pmc11_1 -o p1 -- python3 -u tools/bench_terasort.py --steps 2 --warmup 1 > $OUT/pmc11_1.log 2>&1 || exit $?
MR_SORT32_DIGIT_BITS=11 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "onesweep|hist11" --output-format csv -d $OUT/pmc11_2 -o p2 -- python3 -u tools/bench_terasort.py --steps 2 --warmup 1 > $OUT/pmc11_2.log 2>&1 || exit $?
for k in onesweep11 hist11; do
  python3 tools/pmc_summary.py $OUT/pmc11_1 $OUT/pmc11_2 --kernel $k > $OUT/summary_$k.txt 2>&1
done
find $OUT -name "*.csv" -size +20M -delete
