#!/bin/bash
# p0_chain_kernel pooled rows per task (HBK_P0_BAND) on 100k clips: layout line + embed time, twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for b in 6 5 7 6 5 7; do
  echo "== HBK_P0_BAND=$b"
  HBK_P0_BAND=$b HBK_DEBUG_EMBED=1 timeout -k 10 120 python tools/probe_embed.py --clips 100000 --iters 5 --precision split 2>&1 | grep -E "hbk p0 chain|split:" || exit 1
done
