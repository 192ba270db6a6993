#!/bin/bash
# W > 1: the post-map chain on CUs of its own (MR_POST_CUS) — GPU tests, W=8 proxy A/B, rehearsal, trace.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_cumask}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_spmd_dist.py tests/test_sdma_gpu.py tests/test_generic_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 32 0 64; do
    MR_POST_CUS=$v timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_cus$v.r$rep.log 2>&1 || exit $?
    echo "cus=$v rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_w8_cus$v.r$rep.log)"
  done
done
MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_hosttl.log 2>&1 || exit $?
MR_COPY_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_copytl.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cold > $OUT/bench_gpus2.log 2>&1 || exit $?
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/tl -o run -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/tl.log 2>&1
