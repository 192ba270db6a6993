#!/bin/bash
# W=8 per-rank proxy: step time, then the host-side Python profile of the
# same loop (cProfile, cumulative and self time).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-proxy_prof}
mkdir -p $OUT
timeout -k 10 200 python3 tools/proxy_world.py --world 8 --steps 50 > $OUT/proxy_w8.log 2>&1 || exit $?
timeout -k 10 200 python3 -m cProfile -o $OUT/proxy_w8.prof tools/proxy_world.py --world 8 --steps 200 > $OUT/proxy_w8_cprof.log 2>&1 || exit $?
python3 - "$OUT/proxy_w8.prof" > $OUT/proxy_w8_pstats.txt <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
PY
