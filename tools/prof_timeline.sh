#!/bin/bash
# Kernel + memory-copy trace (no PMC) of one program:
#   tools/prof_timeline.sh <outdir-name> <python args...>
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
name=$1; shift
mkdir -p gpurun_out/$name
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/$name -o run -- python3 "$@" > gpurun_out/$name.log 2>&1
