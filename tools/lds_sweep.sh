set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for kb in 40 56 100 156; do
  echo "== LDS $kb KB"
  HBK_EMBED_LDS_KB=$kb HBK_DEBUG_EMBED=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/lds_$kb -o run -- python3 tools/probe_embed.py --precision split --iters 3 > gpurun_out/lds_$kb.log 2>&1 || { tail -5 gpurun_out/lds_$kb.log; exit 1; }
  grep -E "split chain|split:" gpurun_out/lds_$kb.log | tail -3
  python3 - "$kb" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/lds_{sys.argv[1]}/run_kernel_stats.csv")):
    if 'chain' in r['Name']: print("  ", r['Name'][25:70], r['Calls'], round(float(r['AverageNs'])/1e6, 3))
PY
done
