#!/bin/bash
# Augment GPU tests (prepare / launch split), then config 5 sequential vs pipelined.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_augment.py tests/test_stages_gpu.py tests/test_placement.py > gpurun_out/ov2_tests.log 2>&1 || { tail -30 gpurun_out/ov2_tests.log; exit 1; }
tail -2 gpurun_out/ov2_tests.log
for pol in ${POLICIES:-off spill:64 spill:48}; do
  echo "=== $pol"
  timeout -k 10 240 python bench.py --config 5 --no-cpu --overlap $pol > gpurun_out/ov2_bench_${pol/:/_}.json 2> gpurun_out/ov2_bench_${pol/:/_}.err || { tail -5 gpurun_out/ov2_bench_${pol/:/_}.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/ov2_bench_${pol/:/_}.json'))
print('$pol', d['value'], d['ms_per_step'], [(r['kernel'][:20], r['ms_per_step']) for r in [d['roofline']]+d['roofline_other']])"
done
