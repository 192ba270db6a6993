#!/bin/bash
# Bigram timeline + repeats; forced-shuffle headline with one / three host waits
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_misc}
mkdir -p $OUT
bash tools/r5_bigram_tl.sh ${1:-r5_misc}/bg || exit $?
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 10 --warmup 2 > $OUT/bigram_$i.log 2>&1 || exit $?
  echo "bigram $(grep -o '"ms_per_step": [0-9.]*' $OUT/bigram_$i.log)"
done
for r in 1 2; do for ss in 1 0; do
  MR_SINGLE_SYNC=$ss timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --force-shuffle > $OUT/fs_ss$ss.r$r.log 2>&1 || exit $?
  echo "fs single_sync=$ss $(grep -o '"force_shuffle_ms_per_step": [0-9.]*' $OUT/fs_ss$ss.r$r.log)"
done; done
