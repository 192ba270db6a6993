#!/bin/bash
# W > 1 post-map work on a high-priority stream (MR_POST_STREAM): single-sync GPU tests,
# W=8 proxy A/B alternating, bench --gpus 2 rehearsal, one traced proxy run.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_post}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spmd_dist.py tests/test_sdma_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 1 0; do
    MR_POST_STREAM=$v timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_post$v.r$rep.log 2>&1 || exit $?
    echo "post=$v rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_w8_post$v.r$rep.log)"
  done
done
MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_hosttl.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cold > $OUT/bench_gpus2.log 2>&1 || exit $?
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/tl -o run -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/tl.log 2>&1
