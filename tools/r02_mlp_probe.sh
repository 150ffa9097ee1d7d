#!/bin/bash
# Train-step probe session: timing, stage trace, SQ counters of the fused kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-p1}
echo "=== timing"
timeout -k 10 120 python tools/probe_mlp.py 200 2>&1 | grep -v amdgpu.ids | tee $OUT/mlp_timing_$TAG.log || exit 1
echo "=== trace"
timeout -k 10 120 python tools/probe_mlp.py --trace 2>&1 | grep -v amdgpu.ids | tee $OUT/mlp_trace_$TAG.log || exit 1
if [ -n "$KSTATS" ]; then
  echo "=== kernel stats"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $OUT/mlp_ks_$TAG -o run -- python3 tools/probe_mlp.py 50 > $OUT/mlp_ks_$TAG.log 2>&1 || { tail -5 $OUT/mlp_ks_$TAG.log; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$OUT/mlp_ks_$TAG/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]: print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
fi
if [ -n "$PMC" ]; then
  echo "=== pmc"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -f csv -d $OUT/mlp_pmc_$TAG -o run -- python3 tools/probe_mlp.py 50 > $OUT/mlp_pmc_$TAG.log 2>&1 || { tail -5 $OUT/mlp_pmc_$TAG.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU -f csv -d $OUT/mlp_pmc2_$TAG -o run -- python3 tools/probe_mlp.py 50 > $OUT/mlp_pmc2_$TAG.log 2>&1 || { tail -5 $OUT/mlp_pmc2_$TAG.log; exit 1; }
fi
echo "=== done"
