#!/bin/bash
# Round-3 general plane: its GPU tests first, then the whole GPU suite, smoke(),
# the 1-GPU bench, and PMC passes of the word-count map kernel
# (tools/gpu_r3_base.sh).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3_gen}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_generic_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_generic.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
bash tools/gpu_r3_base.sh ${1:-r3_gen}
