"""Per-step kernel summary of a bench.py run profiled by rocprofv3, restricted
to the dispatches between bench.py's profiling markers (hbk_profile_mark_kernel,
include/hbk.h): the timed region (tags 1 -> 2) and, when present, the
sequential stage-timing steps (tags 3 -> 4) that bench.py's per-stage
rooflines are measured on. Setup, warmup and teardown dispatches are dropped.

Inputs (any subset; each a rocprofv3 -d directory, searched recursively):
  --trace DIR   rocprofv3 --kernel-trace [--stats]   -> calls and durations
  --fetch DIR   rocprofv3 --pmc FETCH_SIZE           -> HBM read bytes
  --write DIR   rocprofv3 --pmc WRITE_SIZE           -> HBM write bytes
  --sq DIR      rocprofv3 --pmc SQ_... GRBM_GUI_ACTIVE -> MFMA / VALU busy
  --steps K / --stage-steps S: the bench's timed steps and stage steps, to
                normalise per step.

HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (counters in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read,
MI355X_MICROARCH.md §HBM). Busy fractions use the dispatch's own cycles,
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs, ibid. DVFS note):
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * cycles)
  valu_issue = 4 * SQ_INSTS_VALU / (1024 SIMDs * cycles)   (4 cycles per wave64
               VALU instruction; MFMA and transcendental issue counted at 4)
Counter passes serialise dispatches, so the busy fractions are per kernel
running alone on its stream's CUs.

usage: python tools/prof_summary.py --trace D [--fetch D --write D --sq D]
       --steps K [--stage-steps S] --out OUT.json [--config C] [--label TEXT]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

MARK = "hbk_profile_mark_kernel"


def rows(d, pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    """Kernel name without namespaces / argument lists, template args kept."""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)             # argument list
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"^hbk::", "", n)
    return n.strip()


def regions(dispatch_names):
    """Marker dispatch ids in order -> {'stage': (a, b), 'timed': (a, b)}."""
    marks = sorted(int(d) for d, n in dispatch_names.items() if MARK in n)
    if len(marks) == 4:
        return {"stage": (marks[0], marks[1]), "timed": (marks[2], marks[3])}
    if len(marks) == 2:
        return {"timed": (marks[0], marks[1])}
    raise SystemExit(f"expected 2 or 4 {MARK} dispatches, found {len(marks)}")


def in_region(did, reg):
    return reg[0] < did < reg[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--stage-steps", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", type=int)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    per = {"timed": a.steps, "stage": a.stage_steps}
    res = {"label": a.label, "config": a.config, "steps": a.steps, "stage_steps": a.stage_steps,
           "formula": {"hbm_bytes": "(2*FETCH_SIZE + WRITE_SIZE)*1024",
                       "cycles": "GRBM_GUI_ACTIVE/8",
                       "mfma_busy": "SQ_VALU_MFMA_BUSY_CYCLES/(1024*cycles)",
                       "valu_issue": "4*SQ_INSTS_VALU/(1024*cycles)"},
           "regions": {}}
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # region -> kernel -> field

    if a.trace:
        tr = rows(a.trace, "*kernel_trace.csv")
        regs = regions({r["Dispatch_Id"]: r["Kernel_Name"] for r in tr})
        for r in tr:
            did = int(r["Dispatch_Id"])
            for rn, reg in regs.items():
                if in_region(did, reg):
                    k = acc[rn][short(r["Kernel_Name"])]
                    k["calls"] += 1
                    k["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for rn, reg in regs.items():
            ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tr
                  if int(r["Dispatch_Id"]) in reg]
            res["regions"].setdefault(rn, {})["marker_span_ms"] = (max(ts)[0] - min(ts)[1]) / 1e6 if len(ts) == 2 \
                else None

    def counters(d, names):
        cc = rows(d, "*counter_collection.csv")
        regs = regions({r["Dispatch_Id"]: r["Kernel_Name"] for r in cc})
        seen = defaultdict(set)
        for r in cc:
            if r["Counter_Name"] not in names:
                continue
            did = int(r["Dispatch_Id"])
            for rn, reg in regs.items():
                if in_region(did, reg):
                    k = acc[rn][short(r["Kernel_Name"])]
                    k[r["Counter_Name"]] += float(r["Counter_Value"])
                    seen[(rn, short(r["Kernel_Name"]))].add(did)
        for (rn, kn), ids in seen.items():
            acc[rn][kn]["pmc_calls_" + os.path.basename(os.path.normpath(d))] = len(ids)

    if a.fetch:
        counters(a.fetch, {"FETCH_SIZE"})
    if a.write:
        counters(a.write, {"WRITE_SIZE"})
    sq_names = {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
                "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_INSTS_LDS", "SQ_WAVES", "GRBM_GUI_ACTIVE"}
    if a.sq:
        counters(a.sq, sq_names)

    for rn, ks in acc.items():
        n = per[rn] or 1
        out = {}
        for kn, f in sorted(ks.items(), key=lambda kv: -kv[1].get("ns", 0.0)):
            e = {}
            calls = f.get("calls") or max([v for c, v in f.items() if c.startswith("pmc_calls_")], default=0)
            if calls:
                e["calls_per_step"] = calls / n
                e["avg_us"] = round(f["ns"] / calls / 1e3, 3)
                e["us_per_step"] = round(f["ns"] / n / 1e3, 3)
            if "FETCH_SIZE" in f or "WRITE_SIZE" in f:
                hbm = (2.0 * f.get("FETCH_SIZE", 0.0) + f.get("WRITE_SIZE", 0.0)) * 1024.0
                e["hbm_bytes_per_step"] = hbm / n
                if calls:
                    e["hbm_bytes_per_launch"] = hbm / calls
                    if f.get("ns"):
                        e["hbm_gbs"] = round(hbm / f["ns"], 2)
            if f.get("GRBM_GUI_ACTIVE"):
                cyc = f["GRBM_GUI_ACTIVE"] / 8.0
                e["mfma_busy"] = round(f.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc), 4)
                e["valu_issue"] = round(4.0 * f.get("SQ_INSTS_VALU", 0.0) / (1024.0 * cyc), 4)
                for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_VALU_MFMA_BUSY_CYCLES",
                          "SQ_WAVES", "GRBM_GUI_ACTIVE"):
                    if c in f:
                        e[c + "_per_step"] = f[c] / n
            for c, v in f.items():
                if c.startswith("pmc_calls_"):
                    e[c] = v
            out[kn] = e
        res["regions"].setdefault(rn, {})["kernels"] = out
        tot_ns = sum(f.get("ns", 0.0) for f in ks.values())
        res["regions"][rn]["kernel_us_per_step"] = round(tot_ns / n / 1e3, 1)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    for rn in ("stage", "timed"):
        if rn not in res["regions"]:
            continue
        print(f"== {rn}: {res['regions'][rn].get('kernel_us_per_step')} us of kernels per step")
        for kn, e in list(res["regions"][rn]["kernels"].items())[:16]:
            print(f"  {e.get('us_per_step', 0):10.1f} us/step  {e.get('calls_per_step', 0):7.1f} calls  "
                  f"avg {e.get('avg_us', 0):9.2f} us  hbm {e.get('hbm_bytes_per_step', 0) / 1e9:7.3f} GB  "
                  f"mfma {e.get('mfma_busy', 0):.3f} valu {e.get('valu_issue', 0):.3f}  {kn[:60]}")


if __name__ == "__main__":
    main()
