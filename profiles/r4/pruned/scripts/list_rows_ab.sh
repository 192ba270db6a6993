#!/bin/bash
# Value-list inserts: 8 rows per thread with batched key / home-tag loads
# (list_rows_kernel, default) vs one row per thread (MR_LIST_ROWS=0),
# alternating, on the reducefn3 word count.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-list_rows_ab}
mkdir -p $OUT
for i in 1 2; do
  for r in 1 0; do
    MR_LIST_ROWS=$r timeout -k 10 200 python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 \
      --steps 10 --warmup 2 > $OUT/rows${r}_$i.log 2>&1 || exit $?
    echo "list_rows=$r run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/rows${r}_$i.log)"
  done
done
