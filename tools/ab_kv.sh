#!/bin/bash
# Evaluation-pass variants on a 64-CU stream: libraries x HBK_KV_WAVES (kernel averages under rocprofv3).
#   LIBS="libhbk.so libhbk_kvd3.so" WAVES="16 8" bash tools/ab_kv.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LIBS:-libhbk.so}; do
for W in ${WAVES:-16}; do
  rm -rf gpurun_out/abkv
  HBK_KV_WAVES=$W HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abkv -o run -- python3 tools/probe_eval.py 6 --cus=64 > gpurun_out/abkv.log 2>&1 || { tail -5 gpurun_out/abkv.log; exit 1; }
  echo "== $L waves $W: $(grep 'per pass' gpurun_out/abkv.log | cut -c1-60)"
  python3 - gpurun_out/abkv <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kv_gemm" in r["Name"]:
        print("  %-50s calls %5s avg %9.2f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/abkv
done
done
