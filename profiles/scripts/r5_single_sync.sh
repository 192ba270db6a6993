#!/bin/bash
# Round 5: the W>1 iteration with two host waits (MR_SINGLE_SYNC) — GPU tests,
# the W=8 proxy before/after, and a kernel + copy trace of both.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_ss}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_spmd_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
for ss in 0 1; do
  MR_SINGLE_SYNC=$ss timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8_ss$ss.log 2>&1 || exit $?
done
for ss in 0 1; do
  MR_SINGLE_SYNC=$ss timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl_ss$ss -o run -- python3 tools/proxy_world.py --world 8 --steps 40 > $OUT/tl_ss$ss.log 2>&1 || exit $?
done
