#!/bin/bash
# PMC passes of the general plane's combine-insert kernel on the CSV group-by
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4_csvpmc
mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex agg_combine --output-format csv \
    -d $OUT/pmc$i -o run -- python3 tools/bench_generic.py --jobs scores --steps 2 --warmup 1 > $OUT/pmc$i.log 2>&1
done
