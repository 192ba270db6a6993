#!/bin/bash
# Rehearsal of the driver's scaling command on a 1-GPU box: N ranks share
# cuda:0 (collectives over gloo, since RCCL refuses two ranks on one device).
# Exercises the N-rank bench path end to end (rank spawn, split assignment,
# count exchange, all-to-all, per-key validation, JSON line); the times are
# NOT scaling numbers (one GPU, host-copy collectives).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-scale_rehearsal}
mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/torchrun_n2.log 2>&1
timeout -k 10 400 python bench.py --gpus 4 --steps 5 --warmup 2 > $OUT/spawn_n4.log 2>&1
