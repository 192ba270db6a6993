#!/bin/bash
# Lazy result downloads of the exact-order tail: GPU tests, then the bigram
# bench (validated) with and without them.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_lazy}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sdma_gpu.py tests/test_exact_order.py \
  tests/test_generic_gpu.py > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 --validate > $OUT/bigram.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"validated_full": [a-z]*' $OUT/bigram.log
