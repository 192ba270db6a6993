#!/bin/bash
# Result downloads: which runtime settings move the bigram job's large
# device->host copies off blit kernels (kernel trace of each variant).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-d2h_env}
mkdir -p $OUT
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/bench_generic.py --jobs bigram --steps 6 --warmup 2 > $OUT/$tag.log 2>&1 || exit $?
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log) copyBuffer: $(grep -c copyBuffer $OUT/$tag/run_kernel_trace.csv)"
}
run base X=1
run nolargebar ROC_ENABLE_LARGE_BAR=0
run limitwg DEBUG_CLR_LIMIT_BLIT_WG=16
run blit1 GPU_BLIT_ENGINE_TYPE=1
