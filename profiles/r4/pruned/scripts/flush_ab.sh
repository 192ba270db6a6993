#!/bin/bash
# LDS-table flushes with speculative home-slot probes (MR_FLUSH_PROBE=1,
# default) vs every key through the full insert (0): GPU tests of the CSV fold
# and the general plane with the probes on, then CSV group-by and bigram A/B.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-flush_ab}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_csv_fold.py \
  tests/test_generic_gpu.py tests/test_combiner_gpu.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
  for p in 1 0; do
    MR_FLUSH_PROBE=$p timeout -k 10 300 python3 tools/bench_generic.py --jobs scores,bigram --steps 8 --warmup 2 \
      > $OUT/probe${p}_$i.log 2>&1 || exit $?
    echo "probe=$p run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/probe${p}_$i.log | paste -sd' ')"
  done
done
