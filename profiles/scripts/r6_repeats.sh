#!/bin/bash
# Round-6 final numbers: each benchmark repeated on one box (the spread of a
# box, beside the spread between boxes the earlier runs show), every step
# under its own time limit, chained with && — a failing or hung step ends it.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6_repeats}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 &&
  timeout -k 10 200 python3 bench.py --resident --steps 20 --warmup 5 > $OUT/resident_$i.log 2>&1 &&
  timeout -k 10 200 python3 tools/proxy_world.py --world 8 > $OUT/proxy_w8_$i.log 2>&1 &&
  MR_REC_CHUNKS=3 timeout -k 10 200 python3 tools/proxy_terasort.py --world 8 --xgmi-gbs 700 > $OUT/ts_proxy_k3_$i.log 2>&1 &&
  MR_REC_CHUNKS=0 timeout -k 10 200 python3 tools/proxy_terasort.py --world 8 --xgmi-gbs 700 > $OUT/ts_proxy_k0_$i.log 2>&1 &&
  timeout -k 10 200 python3 tools/bench_terasort.py > $OUT/terasort_$i.log 2>&1 &&
  timeout -k 10 300 python3 tools/bench_generic.py --jobs bigram --steps 20 > $OUT/bigram_$i.log 2>&1 &&
  timeout -k 10 300 python3 tools/bench_invidx.py --steps 20 --warmup 2 > $OUT/invidx_$i.log 2>&1 || exit $?
  echo "round $i done"
done
