#!/bin/bash
# Record-plane row gather: LDS-DMA staged (MR_REC_GLDS=1) vs register staged,
# its GPU test first, then TeraSort alternating.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-glds_ab}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_records.py -m gpu \
  > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
  for g in 1 0; do
    MR_REC_GLDS=$g timeout -k 10 200 python3 tools/bench_terasort.py > $OUT/ts_glds${g}_$i.log 2>&1 || exit $?
    echo "glds=$g run $i $(grep -o '"ms_per_step": [0-9.]*\|"valid": [a-z]*' $OUT/ts_glds${g}_$i.log | paste -sd' ')"
  done
done
