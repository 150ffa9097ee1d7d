#!/bin/bash
# Train-step latency for the data-parallel modes: on a 64-CU stream, the stage-1
# mix scaled to the per-rank batch of the reference-faithful "global" mode (1,100 / N for
# N = 8, 4, 2) and 1,100, each with the bucket all-reduce captured into the step graph
# (a one-rank RCCL group: the collective's launch and device cost, not xGMI latency).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for B in 138 275 550 1100; do
  timeout -k 10 200 python3 tools/probe_mlp.py 200 --cus=64 --batch=$B --reduce 2>&1 | grep "us per train" || exit 1
  timeout -k 10 200 python3 tools/probe_mlp.py 200 --cus=64 --batch=$B 2>&1 | grep "us per train" || exit 1
done
