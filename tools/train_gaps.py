"""Idle gaps of the busiest-with-k2 queue (the train stream) in a rocprofv3
--kernel-trace CSV, between bench.py's last two profiling markers (else the last `span` seconds): total idle time and the
largest gap classes by (previous kernel -> next kernel).
usage: python tools/train_gaps.py <trace dir> [span_s]"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
span = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
rows = list(csv.DictReader(open(f)))
qk = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(qk, "0"), r["Kernel_Name"][:40]) for r in rows)
q_k2 = collections.Counter(e[2] for e in ev if "k2_rows" in e[3]).most_common(1)[0][0]
tq = [e for e in ev if e[2] == q_k2]
marks = [e for e in ev if "profile_mark" in e[3]]
if len(marks) >= 2:  # bench.py's markers (3, 4 around the stage steps, then 1, 2): the timed region is the last pair
    tq = [e for e in tq if marks[-2][1] <= e[0] and e[1] <= marks[-1][0]]
else:
    t_end = tq[-1][1]
    tq = [e for e in tq if e[0] >= t_end - int(span * 1e9)]
busy = sum(b - a for a, b, _, _ in tq)
wall = tq[-1][1] - tq[0][0]
gaps = collections.defaultdict(lambda: [0, 0])
for p, n in zip(tq, tq[1:]):
    g = n[0] - p[1]
    if g > 0:
        k = (p[3], n[3]) if g > 3000 else ("(gaps <= 3 us)", "")
        gaps[k][0] += 1
        gaps[k][1] += g
print(f"queue {q_k2}: {len(tq)} kernels, wall {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {(wall - busy) / 1e6:.2f} ms")
for (a, b), (c, g) in sorted(gaps.items(), key=lambda x: -x[1][1])[:20]:
    print(f"  {g / 1e6:8.3f} ms  {c:6d} x  {a:40s} -> {b}")
