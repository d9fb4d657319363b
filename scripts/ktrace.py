#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel_trace.csv (+ memory_copy_trace.csv): kernels from the
last occurrence of a marker kernel onward, with start offset and duration (µs)."""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kstats import short  # noqa: E402

path, marker = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_init"
ev = []
for r in csv.DictReader(open(path)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
mc = path.replace("kernel_trace", "memory_copy_trace")
if os.path.exists(mc):
    for r in csv.DictReader(open(mc)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "memcpy:" + r.get("Direction", "")))
ev.sort()
starts = [i for i, e in enumerate(ev) if e[2] == marker]
i0 = starts[-2] if len(starts) > 1 else 0
i1 = starts[-1] if len(starts) > 1 else len(ev)
t0 = ev[i0][0]
for s, e, n in ev[i0:i1]:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n}")
