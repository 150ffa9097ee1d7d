"""Summarise tools/pmc_mel.sh's counter CSVs: per mel kernel, mean counters per dispatch."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_mel"
for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        m = re.search(r"(mel\w*kernel(<\w+>)?)", r["Kernel_Name"])
        if not m:
            continue
        k = m.group(1) + f" lds={r['LDS_Block_Size']}"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        print(f.split("/")[-2], k, {c: f"{v / n[(k, c)]:.3g}" for c, v in sorted(d.items())})
