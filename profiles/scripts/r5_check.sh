#!/bin/bash
# Round-5 checkpoint: GPU test suite, smoke, headline bench and the W=8 proxy.
#   tools/r5_check.sh OUTDIR [tests|bench|proxy ...]   (default: all three)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r5_check}
shift
mkdir -p $OUT
WHAT="${*:-tests bench proxy}"
for w in $WHAT; do
  case $w in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $? ;;
    bench)
      timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_staged.log 2>&1 || exit $? ;;
    proxy)
      timeout -k 10 200 python -u tools/proxy_world.py --world 8 --steps 40 > $OUT/proxy_w8.log 2>&1 || exit $? ;;
    *) echo "unknown step $w"; exit 2 ;;
  esac
done
