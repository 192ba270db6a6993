#!/bin/bash
# Round-4 closing run: the GPU test suite and smoke, kernel statistics of
# every workload on the final tree, then counters (one group per run) of the round's new kernels: the
# fused CSV fold and the text token scan.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r4_end}
mkdir -p $OUT
# first the whole GPU test suite and the smoke run on this tree
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
ks() {  # tag cmd...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$tag -o run -- "$@" \
    > $OUT/ks_$tag.log 2>&1 || exit $?
}
ks staged python3 bench.py --steps 10 --warmup 3 --no-cold
ks resident python3 bench.py --steps 10 --warmup 3 --no-cold --resident
ks scores python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 2
ks wcgen python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 5 --warmup 2
ks invidx python3 tools/bench_invidx.py --steps 5 --warmup 2
ks terasort python3 tools/bench_terasort.py --steps 3 --warmup 1
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "csv_fold|text_emit" --output-format csv \
    -d $OUT/pmc_$i -o run -- python3 tools/bench_generic.py --jobs scores --steps 2 --warmup 1 > $OUT/pmc_$i.log 2>&1 || exit $?
done
