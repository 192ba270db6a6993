#!/bin/bash
# Bigram A/B: result downloads by the runtime's blit vs our copy kernel on a
# few workgroups (MR_D2H_BLOCKS), and span inserts without the LDS combine
# (MR_AGG_DIRECT); the word-count headline with the download knob too.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bigram_ab}
mkdir -p $OUT
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 > $OUT/$tag.log 2>&1 || exit $?
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"
}
run base MR_D2H_BLOCKS=0
run d2h64 MR_D2H_BLOCKS=64
run d2h256 MR_D2H_BLOCKS=256
run direct MR_AGG_DIRECT=1
run d2h64_direct MR_D2H_BLOCKS=64 MR_AGG_DIRECT=1
for b in 0 64; do
  MR_D2H_BLOCKS=$b timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/wc_d2h$b.log 2>&1 || exit $?
  echo "wc d2h$b $(tail -1 $OUT/wc_d2h$b.log | grep -o '"ms_per_step": [0-9.]*')"
done
