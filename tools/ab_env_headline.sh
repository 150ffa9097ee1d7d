#!/bin/bash
# Headline A/B of one environment knob at the driver's settings (partition times), alternating:
#   VAR=HBK_EVAL_CUS VALUES="0 256" ROUNDS=2 bash tools/ab_env_headline.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for V in $VALUES; do
    env "$VAR=$V" HBK_BENCH_PARTITION=1 timeout -k 10 400 python bench.py --other-configs= --no-cpu > $OUT/abe_${V}_${r}.json 2> $OUT/abe_${V}_${r}.err \
      || { tail -20 $OUT/abe_${V}_${r}.err; exit 1; }
    echo "$VAR=$V: $(python3 -c "import json; d=json.loads(open('$OUT/abe_${V}_${r}.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])") | $(grep -h 'partition' $OUT/abe_${V}_${r}.err | tr '\n' ' ')"
  done
done
