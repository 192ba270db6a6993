#!/bin/bash
# Counters of the token scan kernel (text_emit, n-gram mode) on the bigram
# job, one counter group per run.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-text_pmc}
mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "text_emit|text_count" --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 tools/bench_generic.py --jobs bigram --steps 2 --warmup 1 > $OUT/pmc_$i.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- \
  python3 tools/bench_generic.py --jobs bigram --steps 4 --warmup 2 > $OUT/ks.log 2>&1 || exit $?
