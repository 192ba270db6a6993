#!/bin/bash
# Run GPU steps one after another, each under its own time limit, with the
# output of step NAME in OUTDIR/NAME.log:
#
#   tools/run_steps.sh OUTDIR NAME SECONDS 'command' [NAME SECONDS 'command' ...]
#
# A step that fails its checks (exit 1-3: a failed test, a wrong answer) is
# recorded and the next step runs; a step that times out, aborts, faults or is
# killed (exit >= 4: 124/137 time limit, 134 abort, 139 segfault, ...), or whose
# log reports a GPU memory fault (a test's child process that faulted), ends
# the chain there — nothing more touches the GPU after it.
set -u
out=$1
shift
mkdir -p "$out"
status=0
while [ $# -ge 3 ]; do
  name=$1 secs=$2 cmd=$3
  shift 3
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc $(( $(date +%s) - start ))s" | tee -a "$out/steps.txt"
  if [ $rc -ne 0 ] && grep -qiE "illegal memory access|hipErrorIllegalAddress|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|unspecified launch failure" "$out/$name.log"; then
    # a failed test or check whose log shows a GPU fault: the card may be left
    # faulted, nothing more runs on it
    echo "step $name hit a GPU fault (rc=$rc): no further GPU steps" | tee -a "$out/steps.txt"
    exit 5
  fi
  if [ $rc -ne 0 ]; then
    status=$rc
    if [ $rc -ge 4 ]; then
      echo "step $name ended with $rc: no further GPU steps" | tee -a "$out/steps.txt"
      exit $rc
    fi
  fi
done
exit $status
