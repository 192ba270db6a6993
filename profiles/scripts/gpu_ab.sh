#!/bin/bash
# A/B of an env switch on the 8/4-rank proxies: tools/gpu_ab.sh VAR valA valB
set -e
mkdir -p gpurun_out
V=$1; A=$2; B=$3
for rep in 1 2; do for val in $A $B; do for w in 8 4; do
  env $V=$val timeout -k 10 120 python -u tools/proxy_world.py --world $w --steps 30 > gpurun_out/ab_${V}_${val}_w${w}_r$rep.log 2>&1
done; done; done
