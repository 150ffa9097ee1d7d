#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of a probe script whose
# kernels match PATTERN: bash tools/prof_probe.sh PATTERN script.py [args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
PAT=$1; shift
rm -rf gpurun_out/pp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pp -o run -- python3 "$@" > gpurun_out/pp.log 2>&1 || { tail -5 gpurun_out/pp.log; exit 1; }
grep -v Warn gpurun_out/pp.log | tail -4
f=$(find gpurun_out/pp -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$PAT" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"]:
        print("%-60s calls %5s avg %9.1f us min %9.1f max %9.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                                   float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
rm -rf gpurun_out/pp
