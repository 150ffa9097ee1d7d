#!/bin/bash
# Train-step kernel tests + probe, then the config-5 overlap policies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp_fused_gpu.py tests/test_classifier_gpu.py > gpurun_out/ov_tests.log 2>&1 || { tail -30 gpurun_out/ov_tests.log; exit 1; }
tail -2 gpurun_out/ov_tests.log
timeout -k 10 120 python tools/probe_mlp.py 200 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ov_mlp_timing.log || exit 1
for pol in ${POLICIES:-off prio spill:64 split:64 split:96}; do
  echo "=== $pol"
  timeout -k 10 240 python bench.py --config 5 --no-cpu --overlap $pol > gpurun_out/ov_bench_${pol/:/_}.json 2> gpurun_out/ov_bench_${pol/:/_}.err || { tail -5 gpurun_out/ov_bench_${pol/:/_}.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/ov_bench_${pol/:/_}.json'))
print('$pol', d['value'], d['ms_per_step'], [(r['kernel'][:20], r['ms_per_step']) for r in [d['roofline']]+d['roofline_other']])"
done
