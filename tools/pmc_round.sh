#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/pmc_probe.sh mel2 python3 tools/probe_mel.py 20000 &&
HBK_MEL_V1=1 bash tools/pmc_probe.sh mel1 python3 tools/probe_mel.py 20000 &&
bash tools/pmc_probe.sh emb python3 tools/probe_embed.py --precision split --iters 1
