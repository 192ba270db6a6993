#!/bin/bash
# Round 5 batch: value-row / tensor-plane / SDMA GPU tests + generic GPU tests, copy-engine
# timeline of the W=8 proxy, bigram with and without SDMA downloads
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_batch1}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_sdma_gpu.py tests/test_value_rows_gpu.py tests/test_digits_spmd.py tests/test_generic_gpu.py tests/test_combiner_gpu.py tests/test_records.py tests/test_mlp_dpsgd.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for mb in 8 0; do
  MR_SDMA_MIN_MB=$mb timeout -k 10 300 python -u tools/bench_generic.py --jobs bigram --steps 8 --warmup 2 --validate > $OUT/bigram_sdma$mb.log 2>&1 || exit $?
done
bash tools/r5_copytl.sh ${1:-r5_batch1}/copytl
