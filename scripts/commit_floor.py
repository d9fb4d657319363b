#!/usr/bin/env python3
"""Write-traffic floor of the S commit in the bit-matrix representation (CPU, from the oracle).

Each new fact (x, a) sets one bit of row x; the commit's write-back is at least one dirty
cache line per distinct (x, line) pair that gets a new bit in a superstep.  This script runs
the CPU oracle on a workload, splits its fact log by superstep (the log is append-only in
superstep order) and counts, per superstep, new facts vs distinct dirty lines of 64 B and
128 B.  Usage: scripts/commit_floor.py [workload] [scale]  ->  JSON on stdout.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from distel_amd import generators  # noqa: E402


def main():
    workload = sys.argv[1] if len(sys.argv) > 1 else "g3"
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ax = generators.workload(workload, scale)
    t0 = time.time()
    o = oracle.saturate(ax, 0)
    sat_s = time.time() - t0
    st = o.stats()
    n = int(o.lib.elo_num_facts(o.ctx))
    x = np.zeros(n, np.uint32)
    a = np.zeros(n, np.uint32)
    import ctypes as C
    p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint32))
    o.lib.elo_copy_log(o.ctx, p(x), p(a), n)
    ds, dl, _ = o.trace()
    o.close()
    init = st["s_init"]
    # row stride in bits: the engine pads a row to 16 B; column = concept id
    words = ((ax.n_concepts + 31) // 32 + 3) // 4 * 4
    out = {"workload": workload, "scale": scale, "concepts": ax.n_concepts, "facts": n, "init": init,
           "oracle_s": round(sat_s, 1), "steps": []}
    pos = n - int(ds.sum())  # the init facts (X, ⊤ and the told closure) come first
    tot = {"new": 0, "words": 0, "lines64": 0, "lines128": 0}
    for t, d in enumerate(ds.tolist()):
        xs, as_ = x[pos:pos + d].astype(np.uint64), a[pos:pos + d].astype(np.uint64)
        pos += d
        bit = xs * (32 * words) + as_
        wd = np.unique(bit >> 5).size
        l64 = np.unique(bit >> 9).size
        l128 = np.unique(bit >> 10).size
        out["steps"].append({"step": t, "new": int(d), "words": int(wd), "lines64": int(l64), "lines128": int(l128)})
        tot["words"] += int(wd)
        tot["new"] += int(d)
        tot["lines64"] += int(l64)
        tot["lines128"] += int(l128)
    out["total"] = tot
    allbits = x.astype(np.uint64) * np.uint64(32 * words) + a.astype(np.uint64)
    out["distinct_words_final"] = int(np.unique(allbits >> np.uint64(5)).size)
    out["distinct_lines64_final"] = int(np.unique(allbits >> np.uint64(9)).size)
    for sh, nm in ((12, "blocks512_final"), (15, "pages4k_final")):
        out[nm] = int(np.unique(allbits >> np.uint64(sh)).size)
    # how far into its row a row's last entry lies (the read-out reads each row up to it)
    last = np.zeros(ax.n_concepts, np.int64)
    np.maximum.at(last, x.astype(np.int64), a.astype(np.int64))
    out["readout_words_to_last_entry"] = int(((last + 32) // 32).sum())
    out["matrix_words"] = int(words) * ax.n_concepts
    out["floor_write_bytes_64"] = 64 * tot["lines64"]
    out["floor_write_bytes_128"] = 128 * tot["lines128"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
