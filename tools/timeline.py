"""Summarise a rocprofv3 --kernel-trace CSV: per queue busy time and the time
both queues were busy at once, over the last part of the run (the timed steps)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
keys = rows[0].keys()
qk = "Queue_Id" if "Queue_Id" in keys else ("Stream_Id" if "Stream_Id" in keys else None)
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(qk, "0"), r["Kernel_Name"][:50]) for r in rows]
ev.sort()
t_end = ev[-1][1]
span = float(sys.argv[2]) if len(sys.argv) > 2 else 0.45  # seconds from the end
t0 = t_end - int(span * 1e9)
ev = [e for e in ev if e[0] >= t0]
queues = sorted(set(e[2] for e in ev))
print("columns:", list(keys)[:12])
print("queues:", queues, "kernels:", len(ev))
# busy intervals per queue (union)
def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out
busy = {q: union([(a, b) for a, b, qq, _ in ev if qq == q]) for q in queues}
tot = ev[-1][1] - ev[0][0]
for q in queues:
    s = sum(b - a for a, b in busy[q])
    names = {}
    for a, b, qq, n in ev:
        if qq == q:
            names[n] = names.get(n, 0) + (b - a)
    top = sorted(names.items(), key=lambda x: -x[1])[:4]
    print(f"queue {q}: busy {s / 1e6:.1f} ms of {tot / 1e6:.1f} ms; top {[(n[:28], round(v / 1e6, 1)) for n, v in top]}")
if len(queues) >= 2:
    a_iv, b_iv = busy[queues[0]], busy[queues[1]]
    i = j = 0
    ov = 0
    while i < len(a_iv) and j < len(b_iv):
        lo, hi = max(a_iv[i][0], b_iv[j][0]), min(a_iv[i][1], b_iv[j][1])
        if hi > lo:
            ov += hi - lo
        if a_iv[i][1] < b_iv[j][1]:
            i += 1
        else:
            j += 1
    print(f"both busy: {ov / 1e6:.1f} ms")
