#!/bin/bash
# Counters of the W = 8 proxy's post-map kernels (one counter group per run, kernel-trace free)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_pmc_w8}
mkdir -p $OUT
RE="cp_|tail_|onesweep|insert_received|wc_map3|offbytes"
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" --output-format csv -d $OUT/pmc_$i -o run -- \
    python3 tools/proxy_world.py --world 8 --steps 10 --warmup 3 > $OUT/pmc_$i.log 2>&1 || exit $?
done
for k in wc_map3 cp_count cp_scan cp_scatter insert_received tail_scatter tail_padhist onesweep tail_offbytes; do
  python3 tools/pmc_summary.py $OUT/pmc_1 $OUT/pmc_2 $OUT/pmc_3 $OUT/pmc_4 --kernel $k > $OUT/summary_$k.txt 2>&1
done
find $OUT -name "*.csv" -size +20M -delete
