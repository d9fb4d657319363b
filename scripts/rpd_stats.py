#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (kernel trace): calls, total / average
duration, sorted by total.  Usage: scripts/rpd_stats.py DB [--csv OUT] [--grep NAME]"""
import argparse
import collections
import glob
import sqlite3
import sys


def load(db):
    c = sqlite3.connect(db)
    t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [x for x in t if x.startswith("rocpd_kernel_dispatch")][0]
    ks = [x for x in t if x.startswith("rocpd_info_kernel_symbol")][0]
    q = f"select k.display_name, d.start, d.end, d.stream_id from {kd} d join {ks} k on d.kernel_id = k.id order by d.start"
    return list(c.execute(q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--grep")
    a = ap.parse_args()
    dbs = glob.glob(a.db, recursive=True) or [a.db]
    rows = load(dbs[0])
    agg = collections.OrderedDict()
    for name, s, e, _ in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        if a.grep and a.grep not in short:
            continue
        g = agg.setdefault(short, [0, 0])
        g[0] += 1
        g[1] += e - s
    tot = sum(v[1] for v in agg.values())
    lines = ["kernel,calls,total_ms,avg_us,pct"]
    for k, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k},{n},{ns / 1e6:.3f},{ns / n / 1e3:.2f},{100 * ns / max(tot, 1):.1f}")
    out = "\n".join(lines)
    print(out)
    if a.csv:
        open(a.csv, "w").write(out + "\n")


if __name__ == "__main__":
    sys.exit(main())
