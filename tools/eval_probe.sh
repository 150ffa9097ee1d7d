#!/bin/bash
# Evaluation-pass kernels: per-pass time on the whole GPU and on 64 CUs, with kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in 0 64; do
  rm -rf gpurun_out/ev$C
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ev$C -o run -- python3 tools/probe_eval.py 10 --cus=$C > gpurun_out/ev$C.log 2>&1 || { tail -5 gpurun_out/ev$C.log; exit 1; }
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
