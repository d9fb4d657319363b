#!/usr/bin/env python3
"""Summarise the PMC passes of scripts/pmc_session.sh into profiles/pmc/<name>.json.

Usage: scripts/pmc_summary.py gpurun_out/TAG OUT.json WORKLOAD

Per kernel: dispatches, Σ FETCH_SIZE / WRITE_SIZE (KB, as rocprofv3 reports them) and the
HBM bytes per dispatch, corrected by the calibration of this engine's access patterns
(profiles/pmc/r03_pmc_calibration.json, scripts/micro/pmc_cal.hip): FETCH_SIZE reports half the
bytes of a coalesced streaming read (×2, as MI355X_MICROARCH.md has it for gfx950) but one 64-B
unit per random 4–8-B load, i.e. per line request (×1); WRITE_SIZE counts 32 B per scattered
4-B store or atomic, 64 B per 64-bit CAS (×1).  Kernels whose reads are random gathers (the
saturation, the set inserts, the told-closure merges) take ×1, streaming kernels ×2; both the
calibrated and the doubled figure are reported, with the raw one.  The source digest of the HIP
file ties the numbers to the build that produced them (bench.py uses them only for that build).
"""

# read pattern per kernel: random gathers (FETCH_SIZE = bytes of the line requests) or
# coalesced streaming (FETCH_SIZE = half the bytes); calibration: r03_pmc_calibration.json
RANDOM_READ = {"k_expand", "k_jobs", "k_commit", "k_commit_told", "k_rehash", "k_level", "k_level_list", "k_relax",
               "k_reloc_move",
               "k_reloc_claim", "k_ximport", "k_clear_logged", "k_init_facts", "k_stats", "k_succ_fill", "k_group_fill"}
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
                     "(bench.py --steps 1 --warmup 0); hbm_bytes_per_dispatch = (f*FETCH_SIZE + WRITE_SIZE)*1024 "
                     "/ dispatches with f = 1 for random-gather kernels and 2 for streaming ones, as calibrated in "
                     "profiles/pmc/r03_pmc_calibration.json (scripts/micro/pmc_cal.hip)",
           "kernels": {}}
    # the HIP runtime the passes ran on (the bench line each pass printed): the system runtime's
    # copies go to an SDMA engine, torch's bundled runtime blits them on the CUs
    # (__amd_rocclr_copyBuffer dispatches in the table come from the bench's own small D2D / D2H
    # copies: counter readbacks, the profiled classification's run-buffer DMAs, not the timed step)
    for log in sorted(glob.glob(os.path.join(tag, "p*.log"))):
        for line in open(log, errors="replace"):
            if line.startswith("{") and '"hip_runtime"' in line:
                try:
                    res["hip_runtime"] = json.loads(line).get("hip_runtime")
                except ValueError:
                    pass
        if "hip_runtime" in res:
            break
    # informational passes (p3: L2 hit/miss, p4: SQ wave/issue cycles), when present
    extra = {c: load(os.path.join(tag, d), c) for d, c in
             (("p3", "TCC_HIT_sum"), ("p3", "TCC_MISS_sum"), ("p4", "SQ_WAVE_CYCLES"),
              ("p4", "SQ_WAIT_ANY"), ("p4", "SQ_ACTIVE_INST_ANY"))}
    for k in sorted(set(fetch) | set(write)):
        nd = max(fetch.get(k, [0, 0])[0], write.get(k, [0, 0])[0])
        fk, wk = fetch.get(k, [0, 0.0])[1], write.get(k, [0, 0.0])[1]
        ff = 1 if k.split("::")[-1] in RANDOM_READ else 2
        row = {"dispatches": nd, "fetch_kb": round(fk, 3), "write_kb": round(wk, 3), "read_pattern":
               "random (FETCH ×1)" if ff == 1 else "streaming (FETCH ×2)",
               "hbm_bytes_per_dispatch": round((ff * fk + wk) * 1024 / nd, 1) if nd else None,
               "doubled_bytes_per_dispatch": round((2 * fk + wk) * 1024 / nd, 1) if nd else None,
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
