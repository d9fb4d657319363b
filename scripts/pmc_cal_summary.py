#!/usr/bin/env python3
"""Summarise the calibration passes of scripts/micro/pmc_cal (FETCH_SIZE and WRITE_SIZE, one
rocprofv3 --pmc pass each) into profiles/pmc/<out>.json: per access pattern, the counter's bytes
per access and per algorithmic byte.

Usage: scripts/pmc_cal_summary.py gpurun_out/TAG OUT.json
(gpurun_out/TAG holds cal.txt — the micro's own output with the access counts — and the pass
directories c1 (FETCH_SIZE) and c2 (WRITE_SIZE).)
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    tag, out = sys.argv[1], sys.argv[2]
    counts = {}
    for line in open(os.path.join(tag, "cal.txt")):
        m = re.match(r"(k_\w+)\s+accesses (\d+) algorithmic_bytes (\d+)\s+([\d.]+) ms\s+([\d.]+) G", line)
        if m:
            counts[m.group(1)] = dict(accesses=int(m.group(2)), bytes=int(m.group(3)), ms=float(m.group(4)),
                                      g_access_per_s=float(m.group(5)))
    fetch = load(os.path.join(tag, "c1"), "FETCH_SIZE")
    write = load(os.path.join(tag, "c2"), "WRITE_SIZE")
    res = {"method": "scripts/micro/pmc_cal.hip: one launch per access pattern over an 8 GB array (past the 256 MiB "
                     "Infinity Cache), every random access on a distinct 128-B line; rocprofv3 --pmc FETCH_SIZE and "
                     "--pmc WRITE_SIZE in separate passes (KB as reported, ×1024)",
           "patterns": {}}
    for k, c in counts.items():
        f = fetch.get(k, [0, 0.0])[1] * 1024
        w = write.get(k, [0, 0.0])[1] * 1024
        res["patterns"][k] = dict(c, fetch_bytes=f, write_bytes=w,
                                  fetch_per_access=round(f / c["accesses"], 3),
                                  write_per_access=round(w / c["accesses"], 3),
                                  fetch_per_alg_byte=round(f / c["bytes"], 4),
                                  write_per_alg_byte=round(w / c["bytes"], 4))
    json.dump(res, open(out, "w"), indent=1)
    for k, p in res["patterns"].items():
        print(f"{k:12s} fetch/access {p['fetch_per_access']:8.2f} B  write/access {p['write_per_access']:8.2f} B  "
              f"fetch/alg {p['fetch_per_alg_byte']:.3f}  write/alg {p['write_per_alg_byte']:.3f}")


if __name__ == "__main__":
    main()
