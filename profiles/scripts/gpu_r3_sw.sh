#!/bin/bash
# Server/worker deployment (the reference's shape): 1 and 4 GPU workers with a
# cProfile of every worker (MR_WORKER_PROFILE), for the per-job host costs.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_sw}
mkdir -p $OUT
for n in 1 4; do
  MR_WORKER_PROFILE=$OUT/prof$n timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
