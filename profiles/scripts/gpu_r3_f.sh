#!/bin/bash
# Round-3 checkpoint 6: server/worker after worker warm-up + lock-free blob
# copies (1/4/8 workers, one profiled run), W=8 per-rank proxy.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_f}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py tests/test_generic_server_worker.py tests/test_long_poll.py -m "gpu or not gpu" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
for n in 1 4 8; do
  timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
MR_WORKER_PROFILE=$OUT/swprof4 timeout -k 10 300 python -u tools/bench_server_worker.py --workers 4 > $OUT/sw4_prof.log 2>&1
timeout -k 10 300 python -u tools/proxy_world.py --world 8 > $OUT/proxy_w8.log 2>&1
