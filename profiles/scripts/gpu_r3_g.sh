#!/bin/bash
# Round-3: inverted-index timeline (kernels + copies) to see what the 6.6 ms
# step waits on beyond the 5.3 ms host->HBM copy.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_g}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_ii -o run -- python3 tools/bench_invidx.py --steps 5 --warmup 2 > $OUT/prof_ii.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_wc -o run -- python3 bench.py --steps 5 --warmup 2 --no-cold > $OUT/prof_wc.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_terasort.py tests/test_records.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_rec.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
