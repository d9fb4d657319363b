"""Diagnostic: candidates vs new facts per superstep of one G2/G3 classification (EL_TRACE_CANDS)."""
import os, sys
sys.path.insert(0, os.getcwd())
os.environ["EL_TRACE_CANDS"] = "1"
from distel_amd import engine, generators
ax = generators.workload(sys.argv[1] if len(sys.argv) > 1 else "g2", 1.0)
eng, st = engine.classify(ax)
print(st, file=sys.stderr)
