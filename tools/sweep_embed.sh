#!/bin/bash
# LDS-budget / weight-placement / occupancy sweep of the split embedding chains (tuning aid).
set -e
out=gpurun_out/sweep_embed.log
: > $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "libhbk.so 78 auto" "libhbk_w3.so 78 auto" "libhbk_w3.so 52 global" "libhbk_w3.so 52 auto" "libhbk_w3.so 40 global"; do
  set -- $cfg
  echo "=== LIB=$1 LDS_KB=$2 WEIGHTS=$3" >> $out
  HBK_LIB=hey-buddy_amd/lib/$1 HBK_EMBED_LDS_KB=$2 HBK_EMBED_WEIGHTS=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sw_$1_$2_$3 -o run -- python3 tools/probe_embed.py --precision split --iters 3 >> $out 2>&1
done
