#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: short kernel name, calls, total ms, avg/max µs."""
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    if "rocprim" in n:
        m = re.search(r"detail::(\w+?)(?:_kernel)?<", n)
        return "rocprim:" + (m.group(1) if m else "?")
    return n.split("(")[0]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in rows:
        print(f"{short(r['Name'])[:48]:48s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:9.3f} ms "
              f"avg {float(r['AverageNs'])/1e3:9.1f} us  max {float(r['MaxNs'])/1e3:9.1f} us  {100*float(r['TotalDurationNs'])/tot:5.1f}%")


if __name__ == "__main__":
    main()
