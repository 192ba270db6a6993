#!/bin/bash
# The pipelined benchmarks over 20 timed steps (bench.py's count): the first
# timed step's map is not overlapped (the last warm-up step starts nothing
# ahead), so short runs weigh it more.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_steps20}
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_invidx.py --steps 20 --warmup 2 --validate > $OUT/invidx.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_generic.py --jobs bigram,scores,wc_general --steps 20 --warmup 2 --validate > $OUT/generic.log 2>&1 || exit $?
for f in $OUT/*.log; do echo "== $f"; grep -o '"metric": "[^"]*"\|"ms_per_step": [0-9.]*\|"validated_full": [a-z]*' $f | tr '\n' ' '; echo; done
