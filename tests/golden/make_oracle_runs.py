"""Regenerate tests/golden/runs/*.json: what the CPU oracle derives on the full-size workloads the
GPU suite checks bit-exactly — the order-independent closure digest (distel_amd.result.set_digest),
the per-kernel event counters, the per-superstep trace and the totals — so the -m gpu tests compare
the engine with these fixtures instead of re-running the oracle (G3 / G3X at full size: 75–140 s of
oracle time per test on the GPU box).  The G3 case is cross-checked against its SHA-256 pin
(closure_digests.txt, which the independent worklist saturator confirmed, pin_report.txt).

    python tests/golden/make_oracle_runs.py [case ...]   (cases: g3, g3x_compat, g3x_elk)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from distel_amd import generators  # noqa: E402
from distel_amd.result import set_digest  # noqa: E402

CASES = {"g3": ("g3", False), "g3x_compat": ("g3x", True), "g3x_elk": ("g3x", False)}

pinned = {}
for line in open(os.path.join(HERE, "closure_digests.txt")):
    f = line.split()
    if len(f) == 4 and not line.startswith("#"):
        pinned[(f[0], float(f[1]))] = (f[2], f[3])
os.makedirs(os.path.join(HERE, "runs"), exist_ok=True)
for case in sys.argv[1:] or sorted(CASES):
    name, compat = CASES[case]
    ax = generators.workload(name)
    o = oracle.saturate(ax, 0, compat_range=compat)
    fx, fa = o.facts()
    lx, lr, ly = o.links()
    if (name, 1.0) in pinned:
        d_in, d_out = pinned[(name, 1.0)]
        assert ax.digest() == d_in, f"{name}: generator output changed"
        h = hashlib.sha256()
        for a in (fx, fa, lx, lr, ly):
            h.update(np.ascontiguousarray(a).tobytes())
        assert h.hexdigest() == d_out, f"{name}: oracle closure differs from the pinned SHA-256"
    rec = {
        "workload": name, "scale": 1.0, "compat_range": compat, "input_sha256": ax.digest(),
        "set_digest": set_digest(fx, fa, lx, lr, ly),
        "stats": o.stats(),
        "events": o.events().tolist(),
        "trace": [t.tolist() for t in o.trace()],
    }
    with open(os.path.join(HERE, "runs", f"{case}.json"), "w") as f:
        json.dump(rec, f)
    print(case, rec["set_digest"], rec["stats"], flush=True)
    o.close()
