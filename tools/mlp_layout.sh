#!/bin/bash
# The train step alone on a 64-CU stream under each train-CU layout (HBK_TRAIN_CU_LAYOUT),
# per-kernel averages under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LAYOUTS:-spread packed-rr}; do
  D=gpurun_out/mlpl_$L
  rm -rf $D
  HBK_TRAIN_CU_LAYOUT=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $D -o run -- python3 tools/probe_mlp.py 200 --cus=64 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  echo "== $L: $(grep 'us per train' $D.log)"
  python3 - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("k1", "k2", "k3", "k4", "k0")):
        print("  %-40s calls %6s avg %7.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf $D
done
