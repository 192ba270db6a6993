#!/bin/bash
# Round-3 checkpoint: the new GPU tests first (general plane, record widths),
# every GPU test, smoke(), the 1-GPU benches (staged with the forced RCCL
# shuffle timed too, resident), TeraSort and the inverted index, the TeraSort
# data-movement probe, kernel stats of the forced-shuffle bench, and PMC
# passes of the word-count map kernel.  Each GPU step under its own limit.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_check}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_streaming.py tests/test_ops_gpu.py tests/test_exactness.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_new.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --force-shuffle > $OUT/bench_staged_fs.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_resident.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
timeout -k 10 300 python -u tools/ts_move_probe.py > $OUT/ts_move.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fs -o run -- python3 bench.py --steps 20 --warmup 3 --force-shuffle --no-cold > $OUT/prof_fs.log 2>&1
timeout -k 10 120 python -u tools/map_cap_ab.py 23 > $OUT/map_cap23.log 2>&1
i=0
for ctr in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE TCC_EA0_ATOMIC_sum" \
  "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex wc_map3 --output-format csv -d $OUT/pmc$i -o run \
    -- python3 tools/map_cap_ab.py 23 > $OUT/pmc$i.log 2>&1
done
