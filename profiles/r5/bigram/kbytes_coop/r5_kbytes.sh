#!/bin/bash
# Wave-cooperative key-byte gather: GPU tests, kernel stats, validated bigram
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_kbytes}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_exact_order.py tests/test_generic_gpu.py tests/test_ops_gpu.py tests/test_e2e_gpu.py tests/test_sdma_gpu.py tests/test_value_rows_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_generic.py --jobs bigram --steps 10 --warmup 2 > $OUT/bigram_prof.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | grep -i "key_bytes"
timeout -k 10 400 python -u tools/bench_generic.py --jobs bigram --steps 20 --warmup 2 --validate > $OUT/bigram20.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"validated_full": [a-z]*' $OUT/bigram20.log | tr '\n' ' '; echo
