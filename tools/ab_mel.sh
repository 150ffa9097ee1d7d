#!/bin/bash
# A/B of the mel kernels on 100 k clips (whole GPU): v4 with 4-wave blocks + prefetch
# (HBK_MEL_V4=1), v4 with 8-wave blocks (HBK_MEL_V4=8), v2 (default); then the mel GPU
# tests on each v4 form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for r in 1 2; do
  echo "v4/4: $(HBK_MEL_V4=1 timeout -k 10 200 python3 tools/probe_mel.py 100000 2>&1 | tail -1)"
  echo "v4/8: $(HBK_MEL_V4=8 timeout -k 10 200 python3 tools/probe_mel.py 100000 2>&1 | tail -1)"
  echo "v2:   $(timeout -k 10 200 python3 tools/probe_mel.py 100000 2>&1 | tail -1)"
done
for V in 1 8; do
  HBK_MEL_V4=$V timeout -k 10 300 python -u -m pytest tests/test_mel.py tests/test_featurizer.py tests/test_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
done
