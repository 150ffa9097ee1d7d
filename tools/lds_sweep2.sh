#!/bin/bash
# chain-2 / tail LDS budget sweep (HBK_EMBED_LDS_KB) on one 16,384-clip chunk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kb in ${KBS:-0 40 52 78 100}; do
  if [ "$kb" = 0 ]; then unset HBK_EMBED_LDS_KB; else export HBK_EMBED_LDS_KB=$kb; fi
  echo "=== LDS budget ${kb} KB (0 = default)"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/lds_$kb -o run -- python3 tools/probe_embed.py --precision split --iters 3 > gpurun_out/lds_$kb.log 2>&1 || { tail -5 gpurun_out/lds_$kb.log; exit 1; }
  grep -E "split chain: (4|9) stages, in (31|6)x" gpurun_out/lds_$kb.log | head -2
  grep "split:" gpurun_out/lds_$kb.log
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/lds_$kb/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'conv_chain' in r['Name'] or 'p0_chain' in r['Name'] or 'p1_chain' in r['Name']: print('  ', r['Name'][30:75], r['Calls'], r['AverageNs'])
"
done
