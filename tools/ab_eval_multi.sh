#!/bin/bash
# The f32 evaluation pools in one launch (HBK_EVAL_MULTI=1, default) against one launch each (=0):
# the evaluation GPU tests, then the headline (driver settings, partition times), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py tests/test_distributed.py tests/test_dp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for r in 1 2; do
  for M in 1 0; do
    HBK_BENCH_PARTITION=1 HBK_EVAL_MULTI=$M timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/ab_evm_${M}_${r}.json 2> $OUT/ab_evm_${M}_${r}.err \
      || { tail -20 $OUT/ab_evm_${M}_${r}.err; exit 1; }
    echo "multi=$M: $(python3 -c "import json; d=json.loads(open('$OUT/ab_evm_${M}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])") | $(grep -h 'partition' $OUT/ab_evm_${M}_${r}.err | tr '\n' ' ')"
  done
done
