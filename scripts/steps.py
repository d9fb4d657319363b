#!/usr/bin/env python3
"""Per-superstep kernel times of one classification from a rocprofv3 kernel trace (CSV or rocpd
database), with the gaps between kernels on the engine stream.  A classification is cut at its
told closure's first kernel (k_start, the head of el_init) up to the next one's: the reset of the
next classification (k_fill, the matrix clear) runs beside the closure on another stream, so a
cut at k_fill (round 4) booked part of the next closure as the last superstep.
Usage: scripts/steps.py gpurun_out/TAG/prof/run_kernel_trace.csv|tr_results.db [classification index]"""
import collections
import csv
import re
import sys

if sys.argv[1].endswith(".db"):
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    from rpd_stats import load

    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e} for n, s, e, _ in load(sys.argv[1])]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if re.search(r"\bk_start\b", r["Kernel_Name"])] + [len(rows)]
seg = rows[idx[which]:idx[which + 1]]
nxt = int(rows[idx[which + 1]]["Start_Timestamp"]) if idx[which + 1] < len(rows) else None


def nm(s):
    m = re.search(r"(k_\w+)", s)
    return m.group(0) if m else "other"


step, table, tot = -1, collections.defaultdict(dict), collections.Counter()
t0, t1 = int(seg[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in seg)
first = {}
for r in seg:
    n = nm(r["Kernel_Name"])
    if n == "k_expand":
        step += 1
        first[step] = int(r["Start_Timestamp"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[n] += d
    if step >= 0:
        table[step][n] = table[step].get(n, 0) + d
cols = ["k_expand", "k_jobs", "k_commit_told", "k_commit", "k_reloc_claim", "k_reloc_move", "k_reloc_commit"]
print("step " + " ".join(f"{c[2:]:>12s}" for c in cols) + "      wall(us)")
pre = (first[0] - t0) / 1e3 if first else 0.0
print(f"init wall {pre:.1f} us")
for s in sorted(table):
    w = ((first[s + 1] if s + 1 in first else t1) - first[s]) / 1e3
    print(f"{s:4d} " + " ".join(f"{table[s].get(c, 0):12.1f}" for c in cols) + f" {w:12.1f}")
last_commit = max((int(r["End_Timestamp"]) for r in seg if nm(r["Kernel_Name"]) == "k_commit"), default=t1)
print("span us %.1f  busy us %.1f" % ((t1 - t0) / 1e3, sum(tot.values())))
if nxt is not None:
    print("last commit -> next k_start us %.1f" % ((nxt - last_commit) / 1e3))
for k, v in tot.most_common():
    print(f"  {k:20s} {v:9.1f}")
