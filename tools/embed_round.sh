#!/bin/bash
# Embedding kernels: GPU parity tests, then per-kernel times of one 16384-clip
# chunk under rocprofv3 for the default plan (p0s) and the banded p0 kernel
# (HBK_EMBED_NO_P0S=1). TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-emb}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_embed.py tests/test_featurizer.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { tail -40 $OUT/${TAG}_tests.log; exit 1; }
  tail -2 $OUT/${TAG}_tests.log
fi
for V in default nop0s; do
  E=""; [ $V = nop0s ] && E="HBK_EMBED_NO_P0S=1"
  rm -rf $OUT/${TAG}_$V
  env $E timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $OUT/${TAG}_$V -o run -- python3 tools/probe_embed.py --precision split --iters 3 > $OUT/${TAG}_$V.log 2>&1 || { tail -5 $OUT/${TAG}_$V.log; exit 1; }
  grep -E "chain|split:" $OUT/${TAG}_$V.log
  find $OUT/${TAG}_$V -name "*kernel_stats.csv" -exec cp {} $OUT/${TAG}_${V}_kernel_stats.csv \;
  python3 - $OUT/${TAG}_${V}_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(s in r["Name"] for s in ("chain", "p0s")):
        print("  %-60s calls %4s avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf $OUT/${TAG}_$V
done
echo "=== done"
