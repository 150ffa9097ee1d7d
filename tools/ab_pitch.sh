#!/bin/bash
# A/B of library builds on hbk_pitch_shift (25,600 clips x 5 per direction): per-kernel averages.
#   LIBS="libhbk.so libhbk_old.so" bash tools/ab_pitch.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LIBS:-libhbk.so}; do
  rm -rf gpurun_out/abp_$L
  HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abp_$L -o run -- python3 tools/probe_pitch.py 25600 5 > gpurun_out/abp_$L.log 2>&1 || { tail -5 gpurun_out/abp_$L.log; exit 1; }
  echo "== $L: $(grep 'us/clip' gpurun_out/abp_$L.log | tr '\n' ' ')"
  python3 - gpurun_out/abp_$L <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "ps_" in r["Name"]:
        print("  %-44s calls %5s avg %9.2f us" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/abp_$L
done
