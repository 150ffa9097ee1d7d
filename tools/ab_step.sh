#!/bin/bash
# A/B of the train step under environment variants (per-kernel averages from
# rocprofv3 --kernel-trace --stats, and the graph-replayed step time):
#   VARIANTS="HBK_STEP=1 HBK_STEP=2" CUS="64" BATCH=1100 bash tools/ab_step.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CUS:-64}; do
for V in ${VARIANTS:-HBK_STEP=2}; do
  T=gpurun_out/abs_$(echo "$V" | tr '=,' '__')_$C
  rm -rf $T
  env $(echo "$V" | tr ',' ' ') timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $T -o run -- python3 tools/probe_mlp.py ${STEPS:-200} --cus=$C --batch=${BATCH:-1100} > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  echo "== $V ($C CUs; 0 = all; B=${BATCH:-1100}): $(grep 'us per train' $T.log)"
  python3 - $T <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("k1a", "k1s", "k1b", "k1c", "k2_", "k3_", "k3s", "k4_")):
        print("  %-40s calls %6s avg %7.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf $T
done
done
