#!/bin/bash
# Kernel-trace the headline in both NaN-row modes (HBK_NAN_INPLACE=1 / 0) and list per-kernel
# average durations side by side, to attribute the featurize-stream difference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for M in 1 0; do
  rm -rf $OUT/pn$M
  HBK_NAN_INPLACE=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pn$M -o run -- \
    python3 bench.py --other-configs= --no-cpu --steps 6 --warmup 2 > $OUT/pn$M.json 2> $OUT/pn$M.err \
    || { tail -20 $OUT/pn$M.err; exit 1; }
done
python3 - <<'PY'
import csv, glob
rows = {}
for m in ("1", "0"):
    f = glob.glob(f"gpurun_out/pn{m}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        rows.setdefault(r["Name"][:70], {})[m] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
tot = {m: sum(v[m][1] for v in rows.values() if m in v) for m in "10"}
print("total kernel ms: inplace %.1f gather %.1f" % (tot["1"], tot["0"]))
for k, v in sorted(rows.items(), key=lambda kv: -max(x[1] for x in kv[1].values())):
    a, b = v.get("1", (0, 0.0)), v.get("0", (0, 0.0))
    print("%-70s %5d %9.2f | %5d %9.2f" % (k, a[0], a[1], b[0], b[1]))
PY
rm -rf $OUT/pn1 $OUT/pn0
