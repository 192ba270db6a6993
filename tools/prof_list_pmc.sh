#!/bin/bash
# Counters of the value-list insert (agg_insert_kernel) and the posting sort
# on the reducefn3 word count, one counter group per run; kernel statistics.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-list_pmc}
mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "agg_insert|onesweep" --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 2 \
    --warmup 1 > $OUT/pmc_$i.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- \
  python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 2 > $OUT/ks.log 2>&1 || exit $?
