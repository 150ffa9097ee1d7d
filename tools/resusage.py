"""Per-kernel VGPR / AGPR / spill / LDS / occupancy summary from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin); optional name filter args."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[1:]
for r in rows:
    if flt and not any(f in r["name"] for f in flt):
        continue
    print("%-60s VGPR %4s AGPR %3s occ %s spillV %s spillS %s LDS %s" % (
        r["name"][:60], r.get("VGPRs"), r.get("AGPRs"), r.get("Occupancy [waves/SIMD]"),
        r.get("VGPRs Spill"), r.get("SGPRs Spill"), r.get("LDS Size [bytes/block]")))
