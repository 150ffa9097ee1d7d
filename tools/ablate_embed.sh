#!/bin/bash
# Phase ablation of the split embedding chains (libhbk_ablate.so; outputs are
# not meaningful, only the kernel times): HBK_DEBUG_SKIP bits 0 stages,
# 1 im2col, 2 store, 3 staging.
set -e
out=gpurun_out/ablate_embed.log
: > $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sk in 0 1 2 4 8 14 15; do
  echo "=== SKIP=$sk" >> $out
  HBK_LIB=hey-buddy_amd/lib/libhbk_ablate.so HBK_DEBUG_SKIP=$sk timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab_$sk -o run -- python3 tools/probe_embed.py --precision split --iters 3 >> $out 2>&1
done
