#!/bin/bash
# In-place NaN-row fix (HBK_NAN_INPLACE=1, default) against the gather form (=0): the pipeline GPU
# tests, then the headline (driver settings, partition times), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do
  for M in 1 0; do
    HBK_BENCH_PARTITION=1 HBK_NAN_INPLACE=$M timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/ab_nan_${M}_${r}.json 2> $OUT/ab_nan_${M}_${r}.err \
      || { tail -20 $OUT/ab_nan_${M}_${r}.err; exit 1; }
    echo "inplace=$M: $(python3 -c "import json; d=json.loads(open('$OUT/ab_nan_${M}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])") | $(grep -h 'partition' $OUT/ab_nan_${M}_${r}.err | tr '\n' ' ')"
  done
done
