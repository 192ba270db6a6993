#!/bin/bash
# Round-4 checkpoint, part 2: the headline (staged, resident), the general
# plane's jobs (validated), TeraSort and the inverted index.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r4_final}
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --resident > $OUT/bench_resident.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_generic.py --jobs scores,bigram,wc_general --wc-reducers reducefn3 --steps 10 --warmup 2 --validate > $OUT/generic.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1 || exit $?
