"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM
bytes per step (profiles/pmc_*.json, read by bench.py's roofline.traffic).

Each pass must profile ONE bench step (bench.py --steps 1 --warmup 0 --no-cpu
--no-check), FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit
one pass on gfx950). Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the
bytes of a wide coalesced read on gfx950, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024     (counters in KiB)
Usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [CONFIG]
(CONFIG: the bench.py --config the passes ran; bench.py only uses a summary
for the same workload.)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirpath, counter):
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection*.csv"), recursive=True)
    tot = defaultdict(float)
    calls = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                tot[name] += float(row["Counter_Value"])
                calls[name].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return tot, {k: len(v) for k, v in calls.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    config = int(sys.argv[4]) if len(sys.argv) > 4 else None
    fetch, fcalls = load(fdir, "FETCH_SIZE")
    write, _ = load(wdir, "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name, 0.0), write.get(name, 0.0)
        res[name] = {"dispatches": fcalls.get(name, 0), "fetch_kib_raw": f, "write_kib": w,
                     "hbm_bytes_per_step": (2.0 * f + w) * 1024.0}
    with open(out, "w") as fh:
        json.dump({"formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per step (gfx950 FETCH_SIZE = 1/2 bytes)",
                   "config": config, "kernels": res}, fh, indent=1)
    for name, v in res.items():
        if v["hbm_bytes_per_step"] > 1e6:
            print(f"{v['hbm_bytes_per_step'] / 1e9:10.3f} GB  {name[:100]}")


if __name__ == "__main__":
    main()
