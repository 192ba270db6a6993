#!/bin/bash
# Map flush cost breakdown: timing-only ablate modes of config 6 (tools/wc_flush_ablate.py)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-flush}
mkdir -p $OUT
timeout -k 10 300 python -u tools/wc_flush_ablate.py 6 > $OUT/flush_ablate_cfg6.log 2>&1
