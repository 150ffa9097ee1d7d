#!/bin/bash
# Train-partition CU layout A/B (HBK_TRAIN_CU_LAYOUT): the 64 train CUs spread over all 8 XCDs
# (default) against 2 whole XCDs under either mask-bit mapping; headline at driver settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  for L in ${LAYOUTS:-spread packed-rr packed-contig}; do
    HBK_BENCH_PARTITION=1 HBK_TRAIN_CU_LAYOUT=$L timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/ab_cu_${L}_${r}.json 2> $OUT/ab_cu_${L}_${r}.err \
      || { tail -20 $OUT/ab_cu_${L}_${r}.err; exit 1; }
    echo "$L: $(python3 -c "import json; d=json.loads(open('$OUT/ab_cu_${L}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])") | $(grep -h 'partition' $OUT/ab_cu_${L}_${r}.err | tr '\n' ' ')"
  done
done
