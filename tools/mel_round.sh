#!/bin/bash
# mel kernel: GPU parity tests, v1 vs v2 timing on 100k clips, then SQ counters of v2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mel.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mel_tests.log 2>&1 || { tail -30 gpurun_out/mel_tests.log; exit 1; }
tail -3 gpurun_out/mel_tests.log
HBK_MEL_V1=1 timeout -k 10 120 python -u tools/probe_mel.py 100000 || exit 1
timeout -k 10 120 python -u tools/probe_mel.py 100000 || exit 1
if [ -n "$PMC" ]; then
  bash tools/pmc_probe.sh mel2 python3 tools/probe_mel.py 20000 || exit 1
fi
