#!/bin/bash
# list/record planes: GPU tests + module-driven inverted-index and TeraSort benches
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-planes}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_invidx.py tests/test_terasort.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_planes.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --steps 5 --warmup 2 --validate > $OUT/bench_invidx.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py --gb 10 --steps 3 --warmup 1 > $OUT/bench_terasort.log 2>&1
