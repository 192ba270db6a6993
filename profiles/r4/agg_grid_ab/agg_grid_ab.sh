#!/bin/bash
# A/B: workgroup cap of the per-row insert (agg_insert_kernel) on the reducefn3 word count.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-agg_grid_ab}
mkdir -p $OUT
for r in 1 2; do
  for cap in 8192 65536 2048; do
    MR_AGG_INSERT_GRID=$cap timeout -k 10 200 python -u tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 \
      --steps 10 --warmup 2 > $OUT/cap${cap}_$r.log 2>&1 || exit $?
    echo "cap=$cap run $r $(grep -o '"ms_per_step": [0-9.]*' $OUT/cap${cap}_$r.log | tail -1)"
  done
done
