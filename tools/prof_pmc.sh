#!/bin/bash
# One PMC pass per call (no tracing domains): tools/prof_pmc.sh <name> "<counters>" <kernel-regex> <python args...>
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
name=$1; ctr=$2; rx=$3; shift 3
mkdir -p gpurun_out/$name
timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d gpurun_out/$name -o run -- python3 "$@" > gpurun_out/$name.log 2>&1
