#!/bin/bash
# Fused CSV fold ablations: kernel time (rocprofv3 kernel stats) per launch
# shape (MR_CSV_TILES) and per mode (MR_CSV_MODE: 1 = parse only, 2 = no LDS
# combine).  A bench exit of 3 (wrong results, expected in mode 1) is
# accepted; anything else stops the script.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-csv_ab}
mkdir -p $OUT
for cfg in "0 0" "0 1" "0 2" "1 0" "2 0" "4 0" "8 0" "16 0"; do
  set -- $cfg
  tag=t$1_m$2
  MR_CSV_TILES=$1 MR_CSV_MODE=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    --kernel-include-regex csv_fold -d $OUT/$tag -o run -- \
    python3 tools/bench_generic.py --jobs scores --steps 5 --warmup 1 > $OUT/$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "stop: $tag rc=$rc"; exit $rc; fi
  echo "$tag rc=$rc"
done
