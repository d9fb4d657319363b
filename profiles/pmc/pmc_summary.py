#!/usr/bin/env python3
"""Summarise the PMC passes of scripts/pmc_session.sh into profiles/pmc/<name>.json.

Usage: scripts/pmc_summary.py gpurun_out/TAG OUT.json WORKLOAD

Per kernel: dispatches, Σ FETCH_SIZE / WRITE_SIZE (KB, as rocprofv3 reports them) and the
HBM bytes per dispatch, corrected as MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE
reports half the bytes of a wide streaming read (×2), WRITE_SIZE is exact.  The fetch side
of 4–8-byte random accesses is uncalibrated (the guide says so); the doubled figure is
reported and the raw one kept beside it.  The source digest of the HIP file ties the numbers
to the build that produced them (bench.py uses them only for that build).
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(s):
    m = re.search(r"(?:^|::)(k_\w+)\(", s)
    return m.group(1) if m else s.split("(")[0][:48]


def load(pass_dir, counter):
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: [0, 0.0])  # kernel -> [dispatches, Σ value]
    seen = set()
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = kname(r["Kernel_Name"])
            d = (r.get("Dispatch_Id"), k)
            if d not in seen:
                seen.add(d)
                per[k][0] += 1
            per[k][1] += float(r["Counter_Value"])
    return per


def main():
    tag, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = load(os.path.join(tag, "p1"), "FETCH_SIZE")
    write = load(os.path.join(tag, "p2"), "WRITE_SIZE")
    src = open(os.path.join(ROOT, "distel_amd", "csrc", "el_gpu.hip"), "rb").read()
    res = {"workload": workload, "source_sha256": hashlib.sha256(src).hexdigest(),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one classification "
                     "(bench.py --steps 1 --warmup 0); hbm_bytes_per_dispatch = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                     "/ dispatches (gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md 'HBM')",
           "kernels": {}}
    # informational passes (p3: L2 hit/miss, p4: SQ wave/issue cycles), when present
    extra = {c: load(os.path.join(tag, d), c) for d, c in
             (("p3", "TCC_HIT_sum"), ("p3", "TCC_MISS_sum"), ("p4", "SQ_WAVE_CYCLES"),
              ("p4", "SQ_WAIT_ANY"), ("p4", "SQ_ACTIVE_INST_ANY"))}
    for k in sorted(set(fetch) | set(write)):
        nd = max(fetch.get(k, [0, 0])[0], write.get(k, [0, 0])[0])
        fk, wk = fetch.get(k, [0, 0.0])[1], write.get(k, [0, 0.0])[1]
        row = {"dispatches": nd, "fetch_kb": round(fk, 3), "write_kb": round(wk, 3),
               "hbm_bytes_per_dispatch": round((2 * fk + wk) * 1024 / nd, 1) if nd else None,
               "raw_bytes_per_dispatch": round((fk + wk) * 1024 / nd, 1) if nd else None}
        hit, miss = extra["TCC_HIT_sum"].get(k, [0, 0.0])[1], extra["TCC_MISS_sum"].get(k, [0, 0.0])[1]
        if hit + miss:
            row["l2_hit"] = round(hit / (hit + miss), 4)
        wc = extra["SQ_WAVE_CYCLES"].get(k, [0, 0.0])[1]
        if wc:
            row["wait_any_frac"] = round(extra["SQ_WAIT_ANY"].get(k, [0, 0.0])[1] / wc, 4)
            row["active_inst_frac"] = round(extra["SQ_ACTIVE_INST_ANY"].get(k, [0, 0.0])[1] / wc, 4)
        res["kernels"][k] = row
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["kernels"].items():
        print(k, v)


if __name__ == "__main__":
    main()
