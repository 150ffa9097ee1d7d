#!/bin/bash
# embedding kernels: GPU parity tests, then chain timings (p0 pattern kernel vs generic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_embed.py tests/test_featurizer.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/embed_tests.log 2>&1 || { tail -40 gpurun_out/embed_tests.log; exit 1; }
tail -3 gpurun_out/embed_tests.log
HBK_EMBED_NO_P0=1 timeout -k 10 120 python -u tools/probe_embed.py --precision split --iters 3 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/emb_p0 -o run -- python3 tools/probe_embed.py --precision split --iters 3 > gpurun_out/emb_p0.log 2>&1 || { tail -5 gpurun_out/emb_p0.log; exit 1; }
grep -E "p0 chain|split:" gpurun_out/emb_p0.log
