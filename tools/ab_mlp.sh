#!/bin/bash
# A/B of library variants on the train step (64-CU stream): per-kernel averages.
#   LIBS="libhbk.so libhbk_k3d4.so" CUS="64 0" bash tools/ab_mlp.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CUS:-64}; do
for L in ${LIBS:-libhbk.so}; do
  rm -rf gpurun_out/ab_$L
  HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab_$L -o run -- python3 tools/probe_mlp.py 200 --cus=$C > gpurun_out/ab_$L.log 2>&1 || { tail -5 gpurun_out/ab_$L.log; exit 1; }
  echo "== $L ($C CUs; 0 = all): $(grep 'us per train' gpurun_out/ab_$L.log)"
  python3 - gpurun_out/ab_$L <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("k1a", "k1b", "k2_", "k3_", "k4_")):
        print("  %-40s calls %6s avg %7.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/ab_$L
done
done
