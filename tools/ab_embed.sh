#!/bin/bash
# A/B of hbk_embed_clips: the tree's libhbk.so against hey-buddy_amd/lib/libhbk_old.so,
# alternating, 100k clips, split precision.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2; do
  for L in hey-buddy_amd/lib/libhbk.so hey-buddy_amd/lib/libhbk_old.so; do
    echo "== $L"
    HBK_DEBUG_EMBED=0 timeout -k 10 120 python tools/probe_embed.py --clips 100000 --iters 5 --precision split --lib $L 2>&1 | grep "split:" || exit 1
  done
done
