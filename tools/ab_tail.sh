#!/bin/bash
# The embedding's tail on the t3s pipeline against the generic split-f16 kernel
# (HBK_EMBED_NO_T3S=1): hbk_embed_clips on 100k clips, per-kernel averages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in t3s generic; do
  rm -rf gpurun_out/tail_$V
  if [ $V = generic ]; then export HBK_EMBED_NO_T3S=1; else unset HBK_EMBED_NO_T3S; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tail_$V -o run -- python3 tools/probe_embed.py --clips 100000 --iters 3 --precision split > gpurun_out/tail_$V.log 2>&1 || { tail -5 gpurun_out/tail_$V.log; exit 1; }
  echo "== $V: $(grep 'split:' gpurun_out/tail_$V.log)"
  python3 - gpurun_out/tail_$V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(s in r["Name"] for s in ("chain", "gather")):
        print("  %-44s calls %5s avg %9.2f us" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf gpurun_out/tail_$V
done
