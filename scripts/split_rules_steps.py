#!/usr/bin/env python3
"""k_expand time per rule group and superstep from a rocprofv3 trace of a run with
EL_SPLIT_EXPAND=2 (the S role launched once per rule group CR1, CR2, CR3, CR4, rest; then the
link role per rule group CR4 half-2, CR5, CR6, rest; then the activation and propagation roles).  Usage: scripts/split_rules_steps.py DB [classification]"""
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1], recursive=True)[0]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = sqlite3.connect(db)
t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = [x for x in t if x.startswith("rocpd_kernel_dispatch")][0]
ks = [x for x in t if x.startswith("rocpd_info_kernel_symbol")][0]
rows = list(c.execute(f"select k.display_name, d.start, d.end from {kd} d join {ks} k on d.kernel_id = k.id "
                      "order by d.start"))
starts = [i for i, r in enumerate(rows) if "k_start" in r[0]] + [len(rows)]
seg = rows[starts[which]:starts[which + 1]]
cols = ["S:CR1", "S:CR2", "S:CR3", "S:CR4", "S:rest", "L:CR4", "L:CR5", "L:CR6", "L:rest", "jobs", "commit"]
print("step " + " ".join(f"{x:>8s}" for x in cols))
run, jobs, com, k = [], 0.0, 0.0, 0
tot = [0.0] * len(cols)
for name, s, e in seg + [("k_expand", 0, 0)]:
    d = (e - s) / 1e3
    if "k_expand" in name:
        if com > 0 or jobs > 0:  # a new superstep starts
            v = [0.0] * len(cols)
            S = ["S:CR1", "S:CR2", "S:CR3", "S:CR4", "S:rest"]
            L = ["L:CR4", "L:CR5", "L:CR6", "L:rest"]
            lab = S + L if len(run) >= 9 else S if len(run) == 5 else L
            for i, x in enumerate(run):
                v[cols.index(lab[min(i, len(lab) - 1)])] += x
            v[-2], v[-1] = jobs, com
            tot = [a + b for a, b in zip(tot, v)]
            print(f"{k:4d} " + " ".join(f"{x:8.1f}" for x in v))
            k += 1
            run, jobs, com = [], 0.0, 0.0
        if s:
            run.append(d)
    elif "k_jobs" in name:
        jobs += d
    elif "k_commit" in name:
        com += d
print(" sum " + " ".join(f"{x:8.1f}" for x in tot))
