#!/bin/bash
# Downloads by shader stores vs SDMA: staged bench (repeat) and the W=8/W=4 per-rank proxies
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-d2hab2}
mkdir -p $OUT
for r in 1 2; do for m in sdma kernel; do
MR_D2H=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cold > $OUT/staged_${m}_$r.log 2>&1
done; done
for w in 8 4; do for m in sdma kernel; do
MR_D2H=$m timeout -k 10 300 python -u tools/proxy_world.py --world $w --steps 30 > $OUT/proxy_w${w}_$m.log 2>&1
done; done
for m in sdma kernel; do
MR_D2H=$m MR_RESIDENT=1 timeout -k 10 300 python -u tools/proxy_world.py --world 8 --steps 30 > $OUT/proxy_w8_resident_$m.log 2>&1
done
