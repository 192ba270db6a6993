#!/bin/bash
# Counters of the word-count map kernel on the HBM-resident corpus (final round-5 code), two passes
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_map_pmc}
mkdir -p $OUT
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "wc_map3" --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 bench.py --resident --steps 3 --warmup 1 --no-cold > $OUT/pmc_$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT/pmc_1 $OUT/pmc_2 --kernel wc_map3
