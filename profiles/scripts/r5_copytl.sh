#!/bin/bash
# Copy-engine timeline of the W=8 proxy (HIP events on the copy stream), both sync modes
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_copytl}
mkdir -p $OUT
for ss in 1 0; do
  MR_COPY_TIMELINE=1 MR_SINGLE_SYNC=$ss timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_ss$ss.log 2>&1 || exit $?
done
MR_COPY_TIMELINE=1 timeout -k 10 200 python -u tools/proxy_world.py --world 1 --steps 10 > $OUT/proxy_w1.log 2>&1 || exit $?
MR_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/tl -o run -- python3 tools/proxy_world.py --world 8 --steps 30 > $OUT/tl.log 2>&1
