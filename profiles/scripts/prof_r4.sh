#!/bin/bash
# Round-4 profile pass: the word-count map kernel's launch shapes (kernel
# times on the full corpus in HBM + PMC groups for shapes 0 and 1), and
# rocprofv3 kernel statistics of the general plane's jobs (CSV group-by,
# bigram, word count with a batched device reducer).  Counters and kernel
# traces in separate runs; every GPU step under its own limit.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r4_prof}
mkdir -p $OUT
for c in 0 1 3; do
  MR_WC_MAP_CONFIG=$c timeout -k 10 120 python -u tools/map_cap_ab.py 23 > $OUT/map_cap23_c$c.log 2>&1
done
for c in 0 1; do
  i=0
  for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum"; do
    i=$((i+1))
    MR_WC_MAP_CONFIG=$c timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex wc_map3 --output-format csv \
      -d $OUT/pmc_c${c}_$i -o run -- python3 tools/map_cap_ab.py 23 > $OUT/pmc_c${c}_$i.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_scores -o run -- \
  python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 1 > $OUT/ks_scores.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_bigram -o run -- \
  python3 tools/bench_generic.py --jobs bigram --steps 3 --warmup 1 > $OUT/ks_bigram.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_wcgen -o run -- \
  python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 1 > $OUT/ks_wcgen.log 2>&1
