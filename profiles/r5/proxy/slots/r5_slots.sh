#!/bin/bash
# Word-count map LDS footprint (MR_MAP_SLOTS 2048 / 1024): W=8 proxy (post-map kernels beside the next map),
# resident and staged headline, map tests at 1024.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_slots}
mkdir -p $OUT
MR_MAP_SLOTS=1024 timeout -k 10 300 python -u -m pytest tests/test_spmd_dist.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_1024.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 2048 1024; do
    MR_MAP_SLOTS=$v timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_s$v.r$rep.log 2>&1 || exit $?
    echo "slots=$v rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_s$v.r$rep.log)"
  done
done
for v in 2048 1024; do
  MR_MAP_SLOTS=$v timeout -k 10 200 python -u bench.py --resident --steps 20 --warmup 5 --no-cold > $OUT/resident_s$v.log 2>&1 || exit $?
  MR_MAP_SLOTS=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cold > $OUT/staged_s$v.log 2>&1 || exit $?
  echo "slots=$v resident $(tail -1 $OUT/resident_s$v.log | grep -o '"ms_per_step": [0-9.]*') staged $(tail -1 $OUT/staged_s$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
