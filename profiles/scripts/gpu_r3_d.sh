#!/bin/bash
# Round-3 checkpoint 4: exact-order tail fallback + worker native tail tests,
# general-plane bench (bigram, CSV group-by), server/worker at 1/4/8 workers
# and a profiled 4-worker run, TeraSort.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_e2e_gpu.py tests/test_generic_server_worker.py tests/test_generic_gpu.py tests/test_terasort.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 400 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
for n in 1 4 8; do
  timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
MR_WORKER_PROFILE=$OUT/swprof4 timeout -k 10 300 python -u tools/bench_server_worker.py --workers 4 > $OUT/sw4_prof.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
