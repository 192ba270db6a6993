#!/bin/bash
# Repeats of the round-5 headline numbers on one box (run-to-run spread)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_repeats}
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_r$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --resident > $OUT/resident_r$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_r$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/bench_terasort.py > $OUT/terasort_r$r.log 2>&1 || exit $?
  timeout -k 10 400 python -u tools/bench_generic.py --jobs bigram --steps 20 --warmup 2 --validate > $OUT/bigram_r$r.log 2>&1 || exit $?
  echo "r$r staged $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_r$r.log) resident $(grep -o '"ms_per_step": [0-9.]*' $OUT/resident_r$r.log) proxy $(grep -o '"median": [0-9.]*' $OUT/proxy_r$r.log) terasort $(grep -o '"ms_per_step": [0-9.]*' $OUT/terasort_r$r.log) bigram $(grep -o '"ms_per_step": [0-9.]*\|"validated_full": [a-z]*' $OUT/bigram_r$r.log | tr '\n' ' ')"
done
