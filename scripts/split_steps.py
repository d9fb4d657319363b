#!/usr/bin/env python3
"""Per-superstep times of each k_expand / k_commit role from a rocpd kernel trace of a run with
EL_SPLIT_EXPAND=1 EL_SPLIT_COMMIT=1 (one launch per role, in role order: expand S, links,
activations, propagations; commit S, then the other roles).  Supersteps are delimited by
k_commit_told (one per step).  Usage: scripts/split_steps.py DB [classification index]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rpd_stats import load  # noqa: E402

rows = sorted(load(sys.argv[1]), key=lambda r: r[1])
starts = [i for i, r in enumerate(rows) if "k_start" in r[0]] + [len(rows)]
which = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) - 2
seg = rows[starts[which]:starts[which + 1]]
steps, cur = [], []
for name, s, e, _ in seg:
    short = name.replace("(anonymous namespace)::", "").split("(")[0]
    cur.append((short, (e - s) / 1e3))
    if short == "k_commit":  # the last launch of a superstep's commit (other roles)
        steps.append(cur)
        cur = []
print("step  expand-roles(us)                      jobs   told  commit-S  commit-rest")
for k, st in enumerate(steps):
    names = [n for n, _ in st]
    exp = [d for n, d in st if n == "k_expand"]
    jobs = sum(d for n, d in st if n == "k_jobs")
    told = sum(d for n, d in st if n == "k_commit_told")
    com = [d for n, d in st if n == "k_commit"]
    cs = com[0] if len(com) > 1 else 0.0
    cr = com[-1] if com else 0.0
    print(f"{k:4d}  {' '.join(f'{d:8.1f}' for d in exp):36s} {jobs:8.1f} {told:6.1f} {cs:9.1f} {cr:11.1f}")
