#!/bin/bash
# A/B of the k3 split width on the pipelined headline: clips/s and the train
# kernels' HBM bytes per step (FETCH_SIZE / WRITE_SIZE passes over one timed step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for V in narrow wide; do
  E=""; [ $V = wide ] && E="HBK_K3_WIDE=1"
  env $E timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/k3_${V}_bench.json 2> $OUT/k3_${V}_bench.err || { tail -5 $OUT/k3_${V}_bench.err; exit 1; }
  echo "== $V $(cut -c1-200 $OUT/k3_${V}_bench.json | grep -o '"value": [0-9.]*')"
  for P in fetch write; do
    case $P in fetch) CTR=FETCH_SIZE ;; write) CTR=WRITE_SIZE ;; esac
    rm -rf $OUT/k3_${V}_$P
    env $E timeout -k 10 300 rocprofv3 --pmc $CTR -f csv -d $OUT/k3_${V}_$P -o run -- python3 bench.py --steps 1 --warmup 1 --stage-steps 1 --no-cpu --no-check > $OUT/k3_${V}_$P.log 2>&1 || { tail -5 $OUT/k3_${V}_$P.log; exit 1; }
  done
  python3 tools/prof_summary.py --fetch $OUT/k3_${V}_fetch --write $OUT/k3_${V}_write --steps 1 --stage-steps 1 --config 5 --label "k3 $V" --out $OUT/k3_${V}_pmc.json > /dev/null
  python3 - $OUT/k3_${V}_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["regions"]["timed"]["kernels"]
tot = 0
for n, k in d.items():
    if any(s in n for s in ("k1a", "k1b", "k2_rows", "k3_wgrad", "k4_update")):
        b = k.get("hbm_bytes_per_step", 0) / 1000
        tot += b
        print("   %-32s %8.2f MB per train step" % (n[:32], b / 1e6))
print("   train total %.2f MB per train step" % (tot / 1e6))
PY
  rm -rf $OUT/k3_${V}_fetch $OUT/k3_${V}_write
done
