#!/bin/bash
# The generic split-f16 chain kernel on every SE20 chain (pattern kernels off): time per
# 16,384-clip chunk at several LDS budgets per block (HBK_EMBED_LDS_KB; default 78).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HBK_EMBED_NO_P0S=1 HBK_EMBED_NO_P0=1 HBK_EMBED_NO_P1S=1 HBK_EMBED_NO_P1=1 HBK_EMBED_NO_P2S=1 HBK_EMBED_NO_T3S=1
for kb in ${KBS:-78 48 64 100 120 156}; do
  echo "LDS ${kb} KB: $(HBK_EMBED_LDS_KB=$kb timeout -k 10 120 python tools/probe_embed.py --precision split 2>&1 | grep -E '^hbk split chain|^split:' | sed 's/hbk split chain: //' | tr '\n' '|')"
done
