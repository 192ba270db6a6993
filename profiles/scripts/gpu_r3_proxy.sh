#!/bin/bash
# W = 2/4/8 per-rank proxies (loopback collectives) and a kernel trace of the
# W = 8 one: where a rank's share of the step goes at the scaling run's sizes.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_proxy}
mkdir -p $OUT/tl8
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/proxy_world.py --world $w --steps 50 > $OUT/proxy_w$w.log 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl8 -o run -- python3 tools/proxy_world.py --world 8 --steps 20 > $OUT/tl8.log 2>&1
