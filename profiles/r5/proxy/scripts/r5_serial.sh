#!/bin/bash
# W=8 proxy: next map beside the post-map chain vs gated after the tail (MR_SERIAL_MAP), with and without
# CUs reserved for the post-map chain (MR_POST_CUS); single-sync GPU tests with the serial order.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_serial}
mkdir -p $OUT
MR_SERIAL_MAP=1 timeout -k 10 300 python -u -m pytest tests/test_spmd_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_serial.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "0 0" "0 1" "64 0" "64 1" "128 0" "128 1"; do
    set -- $cfg
    MR_POST_CUS=$1 MR_SERIAL_MAP=$2 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_cus$1_serial$2.r$rep.log 2>&1 || exit $?
    echo "cus=$1 serial=$2 rep=$rep $(grep -o '"median": [0-9.]*' $OUT/proxy_cus$1_serial$2.r$rep.log)"
  done
done
MR_SERIAL_MAP=1 MR_HOST_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_serial_hosttl.log 2>&1 || exit $?
MR_SERIAL_MAP=1 MR_COPY_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_serial_copytl.log 2>&1 || exit $?
