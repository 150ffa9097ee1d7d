#!/bin/bash
# Headline (driver settings: --steps 20 --warmup 5) for embed-split settings given as "K:f" args,
# with the partition times (HBK_BENCH_PARTITION=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for kf in "$@"; do
  K=${kf%%:*}; F=${kf##*:}
  HBK_BENCH_PARTITION=1 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu \
      --embed-split $K --embed-split-frac $F > gpurun_out/ss.json 2> gpurun_out/ss.err || { tail -5 gpurun_out/ss.err; exit 1; }
  echo "K=$K f=$F $(grep partition gpurun_out/ss.err | tr '\n' ' ') $(python3 -c 'import json; d=json.loads(open("gpurun_out/ss.json").readline()); print(d["value"], d["ms_per_step"])')"
done
