#!/bin/bash
# Counter passes over tools/probe_mel.py for the current mel kernel and the v2 kernel (HBK_MEL_V2=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mel
rm -rf $OUT && mkdir -p $OUT
A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES"
B="SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for V in v4 v2; do
  if [ $V = v2 ]; then export HBK_MEL_V2=1; unset HBK_MEL_V4; else unset HBK_MEL_V2; export HBK_MEL_V4=1; fi
  for P in a b; do
    CTR=$A; [ $P = b ] && CTR=$B
    timeout -s KILL 90 rocprofv3 --pmc $CTR -f csv -d $OUT/${V}_$P -o run -- \
      python3 tools/probe_mel.py 20000 > $OUT/${V}_$P.log 2>&1 || { tail -20 $OUT/${V}_$P.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_mel/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("::")[-1][:32]
        if "mel" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        print(f.split("/")[2], k, {c: f"{v / n[(k, c)]:.3g}" for c, v in d.items()})
PY
