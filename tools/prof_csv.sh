#!/bin/bash
# CSV group-by (fused CSV fold): kernel + copy trace statistics, then the
# fused kernel's counters (one PMC group per run).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-csv_prof}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- \
  python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 1 > $OUT/ks.log 2>&1
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex csv_fold --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 tools/bench_generic.py --jobs scores --steps 2 --warmup 1 > $OUT/pmc_$i.log 2>&1
done
