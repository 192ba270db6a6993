#!/bin/bash
# TeraSort: the next iteration's map + key sort during this one's row gather (record-plane pipeline)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_ts_ahead}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_terasort.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_terasort.py --steps 10 > $OUT/ts_ahead.r$r.log 2>&1 || exit $?
  echo "ahead $(grep -o '"ms_per_step": [0-9.]*\|"valid": [a-z]*' $OUT/ts_ahead.r$r.log | tr '\n' ' ')"
  MR_PIPELINE=0 timeout -k 10 300 python -u tools/bench_terasort.py --steps 10 > $OUT/ts_plain.r$r.log 2>&1 || exit $?
  echo "plain $(grep -o '"ms_per_step": [0-9.]*\|"valid": [a-z]*' $OUT/ts_plain.r$r.log | tr '\n' ' ')"
done
