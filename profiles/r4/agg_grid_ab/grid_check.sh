#!/bin/bash
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/grid_check
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_generic.py --jobs scores,bigram,wc_general --wc-reducers reducefn3 --steps 10 --warmup 2 --validate > $OUT/generic.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
