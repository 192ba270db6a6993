#!/bin/bash
# Word-count map with the thread's tokens in phases: kernel time, resident bench, word-count GPU tests
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_map_ilp}
mkdir -p $OUT
timeout -k 10 300 python -u tools/map_hot_probe.py > $OUT/probe.log 2>&1 || exit $?
grep "skip packed keys <= 0" $OUT/probe.log
timeout -k 10 300 python -u bench.py --resident --steps 20 --warmup 5 > $OUT/bench_resident.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"per_key_valid": [a-z]*' $OUT/bench_resident.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_e2e_gpu.py tests/test_ops_gpu.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
