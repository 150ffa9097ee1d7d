#!/bin/bash
# Colored-noise fold A/B: the augment GPU tests, then the headline bench with the fold
# (HBK_AUG_COLORED_FOLD=1) and without (=0), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_augment.py tests/test_e2e_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for r in 1 2; do
  for F in 1 0; do
    HBK_AUG_COLORED_FOLD=$F timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/ab_colored_${F}_${r}.json 2> $OUT/ab_colored_${F}_${r}.err \
      || { tail -20 $OUT/ab_colored_${F}_${r}.err; exit 1; }
    echo "fold=$F: $(python3 -c "import json,sys; d=json.loads(open('$OUT/ab_colored_${F}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
  done
done
