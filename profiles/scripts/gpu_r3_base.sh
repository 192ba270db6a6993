#!/bin/bash
# Round-3 entry check: smoke(), the 1-GPU bench (staged and resident), and PMC
# passes of the word-count map kernel (config 6, full corpus in HBM, 2^23-slot
# table as in the resident bench) — one counter group per rocprofv3 run.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_base}
mkdir -p $OUT
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_staged.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_resident.log 2>&1
timeout -k 10 120 python -u tools/map_cap_ab.py 23 > $OUT/map_cap23.log 2>&1
i=0
for ctr in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE TCC_EA0_ATOMIC_sum" \
  "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex wc_map3 --output-format csv -d $OUT/pmc$i -o run \
    -- python3 tools/map_cap_ab.py 23 > $OUT/pmc$i.log 2>&1
done
