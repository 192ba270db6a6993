#!/bin/bash
# Bigram: next map issued right after the exact tail's compaction (1) or after the whole tail (0)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_early}
mkdir -p $OUT
for r in 1 2; do for e in 1 0; do
  MR_EXACT_MAP_EARLY=$e timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 > $OUT/bigram_e$e.r$r.log 2>&1 || exit $?
  echo "early=$e $(grep -o '"ms_per_step": [0-9.]*' $OUT/bigram_e$e.r$r.log)"
done; done
