#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp_fused_gpu.py tests/test_classifier_gpu.py tests/test_onnx_heads.py tests/test_stages_gpu.py > gpurun_out/k2s_tests.log 2>&1 || { tail -30 gpurun_out/k2s_tests.log; exit 1; }
tail -3 gpurun_out/k2s_tests.log
TAG=k2s KSTATS=1 bash tools/r02_mlp_probe.sh
