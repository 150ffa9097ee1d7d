#!/bin/bash
# Evaluation-pass kernels: per-pass time on the whole GPU and on 64 CUs, with kernel stats.
#   LIBS="libhbk.so libhbk_kvab1.so" CUS="64" bash tools/eval_probe.sh   (library A/B; build the ablation with
#   python hey-buddy_amd/build.py --variant=kvab1 --define=HBK_KV_ABLATE=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LIBS:-libhbk.so}; do
for C in ${CUS:-0 64}; do
  echo "== $L, $C CUs (0: all)"
  rm -rf gpurun_out/ev$C
  HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ev$C -o run -- python3 tools/probe_eval.py 10 --cus=$C > gpurun_out/ev$C.log 2>&1 || { tail -5 gpurun_out/ev$C.log; exit 1; }
  grep "per pass" gpurun_out/ev$C.log
  python3 - gpurun_out/ev$C <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("kv_", "k2_rows", "k0_")):
        print("  %-40s calls %6s avg %9.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/ev$C
done
done
