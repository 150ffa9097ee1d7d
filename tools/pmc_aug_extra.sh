#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per run) over the colored-noise and tanh probes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for K in colored tanh; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmcf_$K -o run -- python3 tools/probe_$K.py 20000 > gpurun_out/pmcf_$K.log 2>&1 || { tail -5 gpurun_out/pmcf_$K.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmcw_$K -o run -- python3 tools/probe_$K.py 20000 > gpurun_out/pmcw_$K.log 2>&1 || { tail -5 gpurun_out/pmcw_$K.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmcf_$K gpurun_out/pmcw_$K gpurun_out/pmc_$K.json || exit 1
done
