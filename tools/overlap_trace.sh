#!/bin/bash
# Host enqueue times and a kernel timeline of the overlapped config-5 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
HBK_BENCH_HOSTTIME=1 timeout -k 10 240 python bench.py --config 5 --no-cpu --overlap prio --steps 4 > gpurun_out/ovt.json 2> gpurun_out/ovt.err || { tail -5 gpurun_out/ovt.err; exit 1; }
grep "host ms" gpurun_out/ovt.err
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/ovt_trace -o run -- python3 bench.py --config 5 --no-cpu --overlap prio --steps 3 --warmup 2 > gpurun_out/ovt_trace.log 2>&1 || { tail -5 gpurun_out/ovt_trace.log; exit 1; }
python3 tools/timeline.py gpurun_out/ovt_trace
