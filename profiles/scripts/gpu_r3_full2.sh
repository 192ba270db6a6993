#!/bin/bash
# Round-3 checkpoint after the general-plane / TeraSort work: every GPU test,
# smoke(), the staged / forced-shuffle / resident word-count benches, TeraSort,
# inverted index and the general-plane bench.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_full2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --force-shuffle > $OUT/bench_fs.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_resident.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
timeout -k 10 300 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
