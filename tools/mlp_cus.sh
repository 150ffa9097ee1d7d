set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in 32 64; do
  rm -rf gpurun_out/mlp$C
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/mlp$C -o run -- python3 tools/probe_mlp.py 200 --cus=$C > gpurun_out/mlp$C.log 2>&1 || { tail -5 gpurun_out/mlp$C.log; exit 1; }
  grep "us per train" gpurun_out/mlp$C.log
  python3 - gpurun_out/mlp$C <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("k1", "k2", "k3", "k4", "k0")):
        print("  %-40s calls %6s avg %7.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/mlp$C
done
