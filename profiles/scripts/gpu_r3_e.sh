#!/bin/bash
# Round-3 checkpoint 5: exact-order probe on bigram keys, general-plane bench,
# server/worker at 1/4/8 workers (+ profile), TeraSort, inverted index.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_e}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --force-shuffle > $OUT/bench_fs.log 2>&1
timeout -k 10 300 python -u tools/debug_exact_order.py 30 > $OUT/exact_order.log 2>&1
timeout -k 10 400 python -u tools/bench_generic.py > $OUT/generic.log 2>&1 || true
for n in 1 4 8; do
  timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
MR_WORKER_PROFILE=$OUT/swprof4 timeout -k 10 300 python -u tools/bench_server_worker.py --workers 4 > $OUT/sw4_prof.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1
