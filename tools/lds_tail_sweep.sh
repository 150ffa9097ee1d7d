#!/bin/bash
# Tail-chain kernel time per HBK_EMBED_LDS_KB budget (the generic conv_chain_x3 kernel only runs the
# tail in the default plan): tools/prof_probe.sh over tools/probe_embed.py for each budget given.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for kb in "$@"; do
  echo "== HBK_EMBED_LDS_KB=$kb"
  HBK_EMBED_LDS_KB=$kb bash tools/prof_probe.sh conv_chain tools/probe_embed.py --precision split --iters 3 | grep -v "rocprofv3\|output_stream\|^W\|^E" || exit 1
done
