#!/bin/bash
# LDS / stall counters of the pitch kernels (tools/probe_pitch.py, 25,600 clips):
# one rocprofv3 --pmc pass, summed per kernel by tools/pmc_sq.py-style parsing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_pitch
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -f csv -d $OUT -o run -- python3 tools/probe_pitch.py 25600 1 > $OUT.log 2>&1 || { tail -5 $OUT.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    if "ps_" not in name:
        continue
    parts = name.split("(anonymous namespace)::")
    base = (parts[1] if len(parts) > 1 else name).split("(")[0]
    acc[base][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    print(k, " ".join("%s=%.3g" % (n, v) for n, v in sorted(c.items())))
PY
