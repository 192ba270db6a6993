#!/bin/bash
# Round-3 checkpoint 3: record tests (new tie fix-up), TeraSort + kernel
# stats, server/worker at 1/4/8 workers (unprofiled) + a profiled 4-worker run.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_records.py tests/test_terasort.py tests/test_e2e_gpu.py tests/test_generic_server_worker.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u tools/rec_gather_ab.py > $OUT/rec_gather_ab.log 2>&1
timeout -k 10 300 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ts -o run -- python3 tools/bench_terasort.py > $OUT/prof_ts.log 2>&1
timeout -k 10 400 python -u tools/bench_generic.py > $OUT/generic.log 2>&1
for n in 1 4 8; do
  timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
MR_WORKER_PROFILE=$OUT/swprof4 timeout -k 10 300 python -u tools/bench_server_worker.py --workers 4 > $OUT/sw4_prof.log 2>&1
