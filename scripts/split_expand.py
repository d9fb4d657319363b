#!/usr/bin/env python3
"""k_expand time per rule group from a rocprofv3 trace of a run with EL_SPLIT_EXPAND=2 (the S role
launched once per rule group CR1, CR2, CR3, CR4, rest; then the link, activation and propagation
roles).  Usage: scripts/split_expand.py 'DB glob' [classification index]"""
import collections
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
names = ["S:CR1", "S:CR2", "S:CR3", "S:CR4", "S:rest", "L", "A/P", "A/P"]
tot = collections.Counter()
step, run = [], []
for name, s, e in seg + [("k_commit", 0, 0)]:
    if "k_expand" in name:
        run.append((e - s) / 1e3)
    elif "k_commit" in name or "k_jobs" in name:
        if run:
            labels = names if len(run) >= 5 else ["L", "A/P", "A/P"]
            for i, d in enumerate(run):
                tot[labels[min(i, len(labels) - 1)]] += d
            step.append(run)
            run = []
for k, v in tot.most_common():
    print(f"{k:8s} {v / 1e3:8.3f} ms")
print("supersteps", len(step))
