set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in libhbk.so libhbk_p0sprio1.so libhbk_p0sprio2.so libhbk.so; do
  rm -rf gpurun_out/ab_t
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab_t -o run -- python3 tools/probe_embed.py --precision split --iters 5 --lib hey-buddy_amd/lib/$L > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "== $L $(grep split: gpurun_out/ab.log)"
  python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ab_t/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "chain" in r["Name"]: print("  %-50s %9.1f us" % (r["Name"][:50], float(r["AverageNs"]) / 1e3))
PY
done
rm -rf gpurun_out/ab_t
