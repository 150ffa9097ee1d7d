"""Summarise tools/pmc_probe.sh SQ passes per kernel (mean per dispatch).

usage: python tools/pmc_sq.py gpurun_out/pmc_TAG [kernel-substring ...]
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


def main():
    base = sys.argv[1]
    subs = sys.argv[2:] or [""]
    acc = defaultdict(dict)
    for p in ("a", "b"):
        for k, cs in load(f"{base}_{p}").items():
            for c, v in cs.items():
                acc[k][c] = sum(v) / len(v)
    for k, cs in acc.items():
        if not any(s in k for s in subs):
            continue
        print("==", k[:110])
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:16.4g}")
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM"):
                if c in cs:
                    print(f"   {c + ' / WAVE_CYCLES':42s} {cs[c] / wc:8.3f}")
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS bank conflict / idx active':42s} {cs.get('SQ_LDS_BANK_CONFLICT', 0) / cs['SQ_LDS_IDX_ACTIVE']:8.3f}")


if __name__ == "__main__":
    main()
