#!/bin/bash
# A/B of the mel kernels on 100 k clips (whole GPU): v4 (SoA packed, default) against
# v2 (HBK_MEL_V2=1), then the mel GPU tests on v4 (and v2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for r in 1 2; do
  echo "v4: $(HBK_MEL_V4=1 timeout -k 10 200 python3 tools/probe_mel.py 100000 2>&1 | tail -1)"
  echo "v2: $(HBK_MEL_V2=1 timeout -k 10 200 python3 tools/probe_mel.py 100000 2>&1 | tail -1)"
done
HBK_MEL_V4=1 timeout -k 10 300 python -u -m pytest tests/test_mel.py tests/test_featurizer.py tests/test_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
HBK_MEL_V2=1 timeout -k 10 300 python -u -m pytest tests/test_mel.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
