#!/bin/bash
# Headline A/B of library builds at the driver's settings (partition times), alternating:
#   LIBS="libhbk.so libhbk_old.so" ROUNDS=2 bash tools/ab_lib_headline.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in ${LIBS:-libhbk.so}; do
    HBK_LIB=hey-buddy_amd/lib/$L HBK_BENCH_PARTITION=1 timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/abh_${L}_${r}.json 2> $OUT/abh_${L}_${r}.err \
      || { tail -20 $OUT/abh_${L}_${r}.err; exit 1; }
    echo "$L: $(python3 -c "import json; d=json.loads(open('$OUT/abh_${L}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])") | $(grep -h 'partition' $OUT/abh_${L}_${r}.err | tr '\n' ' ')"
  done
done
