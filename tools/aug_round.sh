#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_augment.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/aug_tests.log 2>&1 || { tail -40 gpurun_out/aug_tests.log; exit 1; }
tail -3 gpurun_out/aug_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/aug_prof -o run -- python3 -u tools/probe_aug.py 100000 > gpurun_out/aug_prof.log 2>&1 || { tail -5 gpurun_out/aug_prof.log; exit 1; }
grep augment: gpurun_out/aug_prof.log
