#!/usr/bin/env python3
"""Every increment of a rocprofv3 kernel trace of the increment leg: from each k_retrigger to the
first k_commit after it (the re-trigger step), the kernels and GPU-idle gaps in between.
Usage: scripts/inc_steps.py DB"""
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from rpd_stats import load  # noqa: E402

rows = [(n.replace("(anonymous namespace)::", "").split("(")[0], s, e, q) for n, s, e, q in
        load(glob.glob(sys.argv[1], recursive=True)[0])]
for k, (n, s, e, q) in enumerate(rows):
    if n != "k_retrigger":
        continue
    j = k + 1
    while j < len(rows) and rows[j][0] != "k_expand":
        j += 1
    c = j
    while c < len(rows) and rows[c][0] != "k_commit":
        c += 1
    print(f"re-trigger at {s / 1e6:.3f} ms: first k_expand {(rows[j][1] - e) / 1e3:.0f} us after it; "
          f"step GPU span {(rows[c][2] - rows[j][1]) / 1e3:.0f} us")
    for n2, s2, e2, q2 in rows[j:c + 1]:
        print(f"   {n2[:40]:40s} start +{(s2 - rows[j][1]) / 1e3:8.0f} us  dur {(e2 - s2) / 1e3:8.0f} us  stream {q2}")
