#!/bin/bash
# Map on a warm vs cold table at W = 8 and 1 shares, PMC counters of the tail compaction
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-probe}
mkdir -p $OUT
timeout -k 10 200 python -u tools/map_warm_probe.py 8 > $OUT/map_warm_w8.log 2>&1
timeout -k 10 200 python -u tools/map_warm_probe.py 1 > $OUT/map_warm_w1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM --kernel-include-regex "tail_compact" --output-format csv -d $OUT/pmc -o c -- python3 tools/map_warm_probe.py 8 > $OUT/pmc.log 2>&1
