#!/bin/bash
# cProfile of the overlapped config-5 bench (host-side enqueue costs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --config 5 --no-cpu --overlap ${POL:-prio} --steps 4 > gpurun_out/hp.json 2> gpurun_out/hp.err || { tail -5 gpurun_out/hp.err; exit 1; }
python -c "
import pstats; p=pstats.Stats('gpurun_out/host.prof'); p.sort_stats('tottime').print_stats(25)" | tail -40
