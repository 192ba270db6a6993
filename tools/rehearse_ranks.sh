#!/bin/bash
# bench.py's multi-rank path rehearsed on ONE GPU: 2 and 4 ranks share the
# card (collectives over gloo there, RCCL on a real node), 5 timed steps.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rehearse}
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python3 bench.py --gpus $n --steps 5 --warmup 2 --no-cold > $OUT/bench_gpus$n.log 2>&1 || exit $?
  echo "gpus=$n $(tail -1 $OUT/bench_gpus$n.log | grep -o '"ms_per_step": [0-9.]*\|"valid": [a-z]*\|"per_key_valid": [a-z]*\|"backend": "[a-z-]*"' | paste -sd' ')"
done
# result downloads: the runtime's blit vs our copy kernel on a few workgroups
# (one system fence per workgroup), bigram (large results) and the headline
for b in 0 16 64; do
  MR_D2H_BLOCKS=$b timeout -k 10 300 python3 tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 > $OUT/bigram_d2h$b.log 2>&1 || exit $?
  echo "bigram d2h=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/bigram_d2h$b.log)"
done
for b in 0 16; do
  MR_D2H_BLOCKS=$b timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cold > $OUT/wc_d2h$b.log 2>&1 || exit $?
  echo "wc d2h=$b $(tail -1 $OUT/wc_d2h$b.log | grep -o '"ms_per_step": [0-9.]*')"
done
