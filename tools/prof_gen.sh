#!/bin/bash
# Kernel statistics (rocprofv3) of the general plane's benches: bigram and the
# reducefn3 word count, a few pipelined steps each.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-gen_prof}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_bigram -o run -- \
  python3 tools/bench_generic.py --jobs bigram --steps 4 --warmup 2 > $OUT/ks_bigram.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_wcgen -o run -- \
  python3 tools/bench_generic.py --jobs wc_general --wc-reducers reducefn3 --steps 4 --warmup 2 > $OUT/ks_wcgen.log 2>&1
