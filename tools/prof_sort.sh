#!/bin/bash
# Radix sort passes on 100 M keys (tools/sort_passes.py) and their kernel stats
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_sort
timeout -k 10 200 python3 tools/sort_passes.py 100000000 > gpurun_out/sort_passes.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sort -o run -- python3 tools/sort_passes.py 100000000 > gpurun_out/prof_sort.log 2>&1
