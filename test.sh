#!/bin/bash
# Integration tests in the reference's style (reference: test.sh): the unit
# tests, then for every storage the four WordCount scenarios run as a real
# server process + worker process, output diffed against the naive oracle.
# (The pytest suite in tests/ covers the same and much more; this script is
# the CLI-level equivalent.)
set -e
cd "$(dirname "$0")"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
export MR_DEFAULT_SLEEP=0.05
python -m lua_mapreduce_1_amd.test
W=lua_mapreduce_1_amd.examples.WordCount
FILES=$(python -c "import $W.taskfn as t; print(' '.join(t.FILES))")
cat $FILES | python -m lua_mapreduce_1_amd.cli.naive | sort > /tmp/mr_naive.$$
port=$((27100 + RANDOM % 1000))
for storage in gridfs shared sshfs; do
  for scenario in combiner nocombiner general single; do
    case $scenario in
      combiner)   mods="$W.taskfn $W.mapfn $W.partitionfn $W.reducefn $W.finalfn $W.reducefn" ;;
      nocombiner) mods="$W.taskfn $W.mapfn $W.partitionfn $W.reducefn $W.finalfn nil" ;;
      general)    mods="$W.taskfn $W.mapfn $W.partitionfn $W.reducefn2 $W.finalfn nil" ;;
      single)     mods="$W $W $W $W $W $W" ;;
    esac
    port=$((port + 1))
    python execute_worker.py 127.0.0.1:$port wc_test --poll 0.05 --max-iter 100 --quiet &
    wpid=$!
    python execute_server.py --sleep 0.3 --poll 0.05 --device host 127.0.0.1:$port wc_test $mods \
      $storage:/tmp/mr_test_st.$$ 2>/dev/null | awk '{print $1,$2}' | sort > /tmp/mr_out.$$
    kill $wpid 2>/dev/null || true
    wait $wpid 2>/dev/null || true
    if diff -q /tmp/mr_out.$$ /tmp/mr_naive.$$ > /dev/null; then
      echo "ok   $storage $scenario"
    else
      echo "FAIL $storage $scenario"; rm -f /tmp/mr_out.$$ /tmp/mr_naive.$$; exit 1
    fi
  done
done
rm -f /tmp/mr_out.$$ /tmp/mr_naive.$$
echo "Ok"
