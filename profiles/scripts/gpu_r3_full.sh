#!/bin/bash
# Round-3 full checkpoint: every GPU test, smoke(), the default bench (staged,
# the driver's shape), the resident bench, TeraSort, inverted index.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --force-shuffle > $OUT/bench_fs.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_resident.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
