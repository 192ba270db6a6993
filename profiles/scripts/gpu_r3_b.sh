#!/bin/bash
# Round-3 checkpoint 2: record spill tier + pruned map kernel tests, resident
# bench, TeraSort kernel stats, server/worker profiles at 1 and 4 workers.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_records.py tests/test_ops_gpu.py tests/test_streaming.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --resident --no-cold > $OUT/bench_resident.log 2>&1
timeout -k 10 300 python -u tools/rec_keys_ab.py > $OUT/rec_keys_ab.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ts -o run -- python3 tools/bench_terasort.py > $OUT/prof_ts.log 2>&1
for n in 1 4; do
  MR_WORKER_PROFILE=$OUT/swprof$n timeout -k 10 300 python -u tools/bench_server_worker.py --workers $n > $OUT/sw$n.log 2>&1
done
