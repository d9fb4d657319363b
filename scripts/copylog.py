"""One small streamed classification with the HIP runtime's log on (AMD_LOG_LEVEL in the
environment): which path its D2H copies take (SDMA vs blit kernel).  GPU diagnostic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (as bench.py: the runtime torch loads)
from distel_amd import engine, generators  # noqa: E402

ax = generators.workload(sys.argv[1] if len(sys.argv) > 1 else "g1", float(sys.argv[2]) if len(sys.argv) > 2 else 0.2)
eng = engine.Engine(device=0)
eng.load(ax)
s = engine.Stream()
for _ in range(2):
    eng.init()
    eng.stream_result(s, release=True)
    eng.saturate()
    eng.result_wait()
print("facts", s.n_facts, "runs", s.n_s_runs, "links", s.n_links, "runs", s.n_l_runs, file=sys.stderr)
