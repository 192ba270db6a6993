#!/bin/bash
# Counters of TeraSort's top kernels on one GPU (row gather, onesweep passes,
# key pass), one counter group per run.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6_ts_pmc}
mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "rec_gather16|onesweep|rec_keys32" \
    --output-format csv -d $OUT/pmc_$i -o run -- python3 tools/bench_terasort.py --steps 2 --warmup 1 \
    > $OUT/pmc_$i.log 2>&1 || exit $?
done
for k in rec_gather16 onesweep rec_keys32; do
  echo "== $k"; python3 tools/pmc_summary.py $OUT/pmc_1 $OUT/pmc_2 $OUT/pmc_3 --kernel $k
done
