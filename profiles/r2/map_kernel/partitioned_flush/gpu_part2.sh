#!/bin/bash
# partitioned flush ablation at 256 and 512 buckets (tools/wc_ablate6.py)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-part2}
mkdir -p $OUT
for nb in 256 512; do for bm in 1 0; do
MR_PART_BUCKET_MAJOR=$bm MR_PART_BUCKETS=$nb timeout -k 10 200 python -u tools/wc_ablate6.py ${@:2} > $OUT/ablate6_nb${nb}_bm$bm.log 2>&1
done; done
