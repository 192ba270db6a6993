#!/bin/bash
# bench.py's multi-rank path (single-sync W > 1 iteration, gloo collectives when ranks share the card)
# rehearsed on ONE GPU at 2 and 4 ranks, then the 1-GPU headline and the W=8 proxy.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_rehearse}
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python3 bench.py --gpus $n --steps 5 --warmup 2 --no-cold > $OUT/bench_gpus$n.log 2>&1 || exit $?
  echo "gpus=$n $(tail -1 $OUT/bench_gpus$n.log | grep -o '"ms_per_step": [0-9.]*\|"valid": [a-z]*\|"per_key_valid": [a-z]*\|"backend": "[a-z-]*"' | paste -sd' ')"
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_1gpu.log 2>&1 || exit $?
for ss in 1 0 1; do
  MR_SINGLE_SYNC=$ss timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 >> $OUT/proxy_w8_ss$ss.log 2>&1 || exit $?
done
MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_hosttl.log 2>&1 || exit $?
MR_COPY_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_copytl.log 2>&1 || exit $?
