"""Diagnostic: per-superstep deltas and the closure digest of a full-size workload, GPU vs the
CPU oracle (python scripts/trace_check.py g3).  Full sizes overflow the first candidate queues;
the deltas must still be the oracle's."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import oracle  # the checker
from distel_amd import engine, generators

w = sys.argv[1] if len(sys.argv) > 1 else "g3"
ax = generators.workload(w, 1.0)
eng, st = engine.classify(ax)
o = oracle.saturate(ax, 0)
same_trace = all(np.array_equal(g, c) for g, c in zip(eng.trace(), o.trace()))
gx, ga = eng.facts()
ox, oa = o.facts()
same_s = np.array_equal(gx, ox) and np.array_equal(ga, oa)
same_l = all(np.array_equal(g, c) for g, c in zip(eng.links(), o.links()))
print(f"{w}: supersteps {st['supersteps']} derived {st['derived']} trace_equal {same_trace} S_equal {same_s} "
      f"R_equal {same_l}")
if not same_trace:
    print("gpu ", [int(v) for v in eng.trace()[0]])
    print("cpu ", [int(v) for v in o.trace()[0]])
sys.exit(0 if (same_trace and same_s and same_l) else 1)
