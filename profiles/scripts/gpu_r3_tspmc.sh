#!/bin/bash
# PMC counters of TeraSort's kernels (one pass per counter group, kernel-trace
# free): bytes fetched / written and wave wait fractions of the onesweep u32
# passes, the row gather and the key pass.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_tspmc}
mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- python3 -u tools/bench_terasort.py --steps 2 --warmup 1 > $OUT/p1.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p2 -o p2 -- python3 -u tools/bench_terasort.py --steps 2 --warmup 1 > $OUT/p2.log 2>&1
for k in onesweep rec_gather16 rec_keys32; do
  python3 tools/pmc_summary.py $OUT/p1 $OUT/p2 --kernel $k > $OUT/summary_$k.txt 2>&1
done
find $OUT -name "*.csv" -size +20M -delete
