#!/bin/bash
# Fused CSV fold ablations: kernel time (rocprofv3 kernel stats) per launch
# shape (MR_CSV_TILES), per mode (MR_CSV_MODE: 1 = parse only, 2 = no LDS
# combine) and per column layout (MR_AGG_ROWS); then the step time of the
# default and of the one-array-per-column layout without the profiler.  A
# bench exit of 3 (wrong results, expected in mode 1) is accepted; anything
# else stops the script.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-csv_ab}
mkdir -p $OUT
for cfg in "0 0 1" "0 0 0" "0 1 1" "0 2 1" "1 0 1" "2 0 1" "4 0 1" "8 0 1"; do
  set -- $cfg
  tag=t$1_m$2_r$3
  MR_CSV_TILES=$1 MR_CSV_MODE=$2 MR_AGG_ROWS=$3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    --kernel-include-regex csv_fold -d $OUT/$tag -o run -- \
    python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 1 > $OUT/$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "stop: $tag rc=$rc"; exit $rc; fi
  echo "$tag rc=$rc"
done
for r in 1 0; do
  MR_AGG_ROWS=$r timeout -k 10 200 python3 tools/bench_generic.py --jobs scores --steps 20 --warmup 3 --validate \
    > $OUT/bench_rows$r.log 2>&1 || exit $?
done
