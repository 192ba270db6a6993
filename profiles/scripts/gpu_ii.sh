#!/bin/bash
# Inverted index: plane tests, validated bench, kernel stats
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ii}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_invidx.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_invidx.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --steps 5 --warmup 2 --validate > $OUT/bench_invidx.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ii -- python3 tools/bench_invidx.py --steps 5 --warmup 2 > $OUT/prof_ii.log 2>&1
