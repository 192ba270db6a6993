#!/bin/bash
# Round-5 final measurements: the headline (staged, resident, forced W>1
# path), the general plane's jobs (validated), TeraSort, the inverted index,
# the server/worker deployment shape and the DP-SGD MLP.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_final}
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --resident > $OUT/bench_resident.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --force-shuffle > $OUT/bench_force_shuffle.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/bench_generic.py --jobs scores,bigram,wc_general --steps 10 --warmup 2 --validate > $OUT/generic.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_terasort.py > $OUT/terasort.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_invidx.py --validate > $OUT/invidx.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_server_worker.py --workers 4 > $OUT/server_worker4.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_mlp.py > $OUT/mlp.log 2>&1 || exit $?
for f in $OUT/*.log; do echo "== $f"; grep -o '"ms_per_step": [0-9.]*\|"valid[a-z_]*": [a-z]*\|"per_key_valid": [a-z]*\|"metric": "[^"]*"' $f | tr '\n' ' '; echo; done
